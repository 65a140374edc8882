/*
 * gfx_image/image.h -- minimal image model for the gfx_imagecompress drop-in.
 *
 * The reference's public header includes "gfx_image/image.h" from the
 * un-vendored al2o3 gfx_image library ("Missing
 * type").  This header supplies the fields the Image_Compress* wrappers touch
 * (width, height, depth, slices, format) plus the pixel storage, and the
 * TinyImageFormat values those wrappers read or produce.  Enum values are this
 * library's own (source-level compatible, not binary-compatible with
 * tiny_imageformat).
 */
#ifndef GFX_IMAGE_IMAGE_H_
#define GFX_IMAGE_IMAGE_H_

#include <stddef.h>
#include <stdint.h>
#include <stdbool.h>

#ifndef AL2O3_EXTERN_C
#ifdef __cplusplus
#define AL2O3_EXTERN_C extern "C"
#else
#define AL2O3_EXTERN_C
#endif
#endif

typedef enum TinyImageFormat {
    TinyImageFormat_UNDEFINED = 0,
    TinyImageFormat_R8_UNORM,
    TinyImageFormat_R8_SNORM,
    TinyImageFormat_R8G8_UNORM,
    TinyImageFormat_R8G8_SNORM,
    TinyImageFormat_R8G8B8_UNORM,
    TinyImageFormat_R8G8B8_SRGB,
    TinyImageFormat_R8G8B8A8_UNORM,
    TinyImageFormat_R8G8B8A8_SRGB,
    TinyImageFormat_R32G32B32A32_SFLOAT,
    TinyImageFormat_DXBC1_RGB_UNORM,
    TinyImageFormat_DXBC1_RGB_SRGB,
    TinyImageFormat_DXBC1_RGBA_UNORM,
    TinyImageFormat_DXBC1_RGBA_SRGB,
    TinyImageFormat_DXBC4_UNORM,
    TinyImageFormat_DXBC4_SNORM,
    TinyImageFormat_DXBC5_UNORM,
    TinyImageFormat_DXBC5_SNORM,
    TinyImageFormat_DXBC7_UNORM,
    TinyImageFormat_DXBC7_SRGB,
    TinyImageFormat_DXBC2_UNORM,
    TinyImageFormat_DXBC2_SRGB,
    TinyImageFormat_DXBC3_UNORM,
    TinyImageFormat_DXBC3_SRGB,
    TinyImageFormat_DXBC6H_UFLOAT,
    TinyImageFormat_DXBC6H_SFLOAT,
    TinyImageFormat_Count
} TinyImageFormat;

typedef struct Image_ImageHeader {
    uint64_t dataSize;   /* bytes at data */
    uint32_t width;
    uint32_t height;
    uint32_t depth;
    uint32_t slices;
    TinyImageFormat format;
    uint32_t flags;
    void *data;          /* host pixels: rows of texels, or rows of 4x4 blocks */
} Image_ImageHeader;

/* Allocate an image whose storage is uninitialised (block formats pad the
 * dimensions up to whole 4x4 blocks, as the reference tests expect 257 -> 260,
 * tests/test_imagecompress.cpp:169-170). */
AL2O3_EXTERN_C Image_ImageHeader const *Image_CreateNoClear(uint32_t width, uint32_t height, uint32_t depth,
                                                            uint32_t slices, TinyImageFormat format);
AL2O3_EXTERN_C Image_ImageHeader const *Image_Create(uint32_t width, uint32_t height, uint32_t depth,
                                                     uint32_t slices, TinyImageFormat format);
AL2O3_EXTERN_C void Image_Destroy(Image_ImageHeader const *image);
AL2O3_EXTERN_C void *Image_RawDataPtr(Image_ImageHeader const *image);

/* Format predicates used by the wrappers. */
AL2O3_EXTERN_C uint32_t TinyImageFormat_ChannelCount(TinyImageFormat fmt);
AL2O3_EXTERN_C bool TinyImageFormat_IsSRGB(TinyImageFormat fmt);
AL2O3_EXTERN_C bool TinyImageFormat_IsSigned(TinyImageFormat fmt);
AL2O3_EXTERN_C bool TinyImageFormat_IsFloat(TinyImageFormat fmt);
AL2O3_EXTERN_C bool TinyImageFormat_IsNormalised(TinyImageFormat fmt);
AL2O3_EXTERN_C bool TinyImageFormat_IsCompressed(TinyImageFormat fmt);
AL2O3_EXTERN_C uint32_t TinyImageFormat_BitSizeOfBlock(TinyImageFormat fmt);

#endif

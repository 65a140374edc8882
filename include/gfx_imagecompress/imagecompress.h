/*
 * imagecompress.h -- drop-in replacement for DeanoC/gfx_imagecompress's public
 * header (reference: include/gfx_imagecompress/imagecompress.h:1-141).
 *
 * Same enums, option structs and entry points.  In this library every
 * Image_CompressAMD* call that does compression work runs the HIP kernels of
 * libgfx_imagecompress_amd.so on the current HIP device; there is no CPU
 * fallback (calls fail -- return NULL or leave `out` untouched -- when no
 * GPU is usable).  Batched device entry points live in gfx_imagecompress_amd/gic.h.
 *
 * Each declaration cites the reference line it replaces.
 */
#pragma once

#include "gfx_image/image.h"

typedef bool (*Image_CompressProgressFunc)(void *user, float percentage);   /* ref :5 */

typedef enum Image_CompressType {                                           /* ref :7-26 */
    Image_CT_None = 0,
    Image_CT_DXBC1,
    Image_CT_DXBC2,
    Image_CT_DXBC3,
    Image_CT_DXBC4,
    Image_CT_DXBC5,
    Image_CT_DXBC6H,
    Image_CT_DXBC7,
    Image_CT_ETC_RGB,
    Image_CT_ETC2_RGB,
    Image_CT_ETC_RGBA_Explicit,
    Image_CT_ETC_RGBA_Interpolated,
    Image_CT_ASTC,
    Image_CT_MAX
} Image_CompressType;

typedef enum Image_CompressPickFlags {                                      /* ref :28-33 */
    Image_CPF_AllowDXBC1to5 = 0x1,
    Image_CPF_AllowASTC = 0x2,
    Image_CPF_AllowETC = 0x8,
    Image_CPF_AllowDXBC6and7 = 0x10
} Image_CompressPickFlags;

typedef struct Image_CompressBC1Options {                                   /* ref :35-38 */
    bool UseAlpha;          /* default false */
    uint8_t AlphaThreshold; /* default 128 */
} Image_CompressBC1Options;

typedef struct Image_CompressAMDBackendOptions {                            /* ref :40-45 */
    bool b3DRefinement;          /* default false (true: Refine3D, BC1/BC2/BC3) */
    bool AdaptiveColourWeights;  /* default false (true: unsupported, call fails) */
    uint8_t RefinementSteps;     /* default 1 */
    uint8_t ModeMask;            /* default 0xFF (BC7) */
} Image_CompressAMDBackendOptions;

typedef struct Image_CompressRichGel99BackendOptions {                     /* ref :47-50 */
    bool perceptual;
    bool fast;
} Image_CompressRichGel999BackendOptions;

/* ref :57-58.  Reference-counted global state; here they only make sure the
 * device tables are resident. */
AL2O3_EXTERN_C void Image_CompressInit(void);
AL2O3_EXTERN_C void Image_CompressDeinit(void);

/* ref :60-62 */
AL2O3_EXTERN_C Image_ImageHeader const *ImageCompress_Compress(Image_CompressType type, bool fast,
                                                                Image_ImageHeader const *src);
/* ref :64-65 */
AL2O3_EXTERN_C Image_CompressType ImageCompress_PickCompressionType(Image_CompressPickFlags flags,
                                                                    Image_ImageHeader const *src);

/* Image level, ref :69-100.  NULL option pointers mean the defaults. */
AL2O3_EXTERN_C Image_ImageHeader const *Image_CompressAMDBC1(Image_ImageHeader const *src,
                                                             Image_CompressAMDBackendOptions const *amdOptions,
                                                             Image_CompressBC1Options const *options,
                                                             Image_CompressProgressFunc progressCallback,
                                                             void *userCallbackData);
AL2O3_EXTERN_C Image_ImageHeader const *Image_CompressAMDBC2(Image_ImageHeader const *src,
                                                             Image_CompressAMDBackendOptions const *amdOptions,
                                                             Image_CompressProgressFunc progressCallback,
                                                             void *userCallbackData);
AL2O3_EXTERN_C Image_ImageHeader const *Image_CompressAMDBC3(Image_ImageHeader const *src,
                                                             Image_CompressAMDBackendOptions const *amdOptions,
                                                             Image_CompressProgressFunc progressCallback,
                                                             void *userCallbackData);
AL2O3_EXTERN_C Image_ImageHeader const *Image_CompressAMDBC4(Image_ImageHeader const *src,
                                                             Image_CompressProgressFunc progressCallback,
                                                             void *userCallbackData);
AL2O3_EXTERN_C Image_ImageHeader const *Image_CompressAMDBC5(Image_ImageHeader const *src,
                                                             Image_CompressProgressFunc progressCallback,
                                                             void *userCallbackData);
AL2O3_EXTERN_C Image_ImageHeader const *Image_CompressAMDBC6H(Image_ImageHeader const *src,
                                                              Image_CompressAMDBackendOptions const *amdOptions,
                                                              Image_CompressProgressFunc progressCallback,
                                                              void *userCallbackData);
AL2O3_EXTERN_C Image_ImageHeader const *Image_CompressAMDBC7(Image_ImageHeader const *src,
                                                             Image_CompressAMDBackendOptions const *amdOptions,
                                                             Image_CompressProgressFunc progressCallback,
                                                             void *userCallbackData);
AL2O3_EXTERN_C Image_ImageHeader const *Image_CompressRichGel999BC7(
    Image_ImageHeader const *src, Image_CompressRichGel999BackendOptions const *richOptions,
    Image_CompressProgressFunc progressCallback, void *userCallbackData);

/* Block level, ref :111-136.  Inputs are normalised floats (0..1). */
AL2O3_EXTERN_C void Image_CompressAMDRGBSingleModeBlock(float const input[4 * 4 * 3], bool adaptiveColourWeights,
                                                        bool b3DRefinement, uint8_t refinementSteps, void *out);
AL2O3_EXTERN_C void Image_CompressAMDAlphaSingleModeBlock(float const input[4 * 4], void *out);
AL2O3_EXTERN_C void Image_CompressAMDExplictAlphaSingleModeBlock(float const input[4 * 4], void *out);
AL2O3_EXTERN_C void Image_CompressAMDBC1Block(float const input[4 * 4 * 4], bool adaptiveColourWeight,
                                              bool b3DRefinement, uint8_t refinementSteps, float alphaThreshold,
                                              void *out);
AL2O3_EXTERN_C void Image_CompressAMDMultiModeLDRBlock(float const input[4 * 4 * 4], uint8_t modeMask,
                                                       bool srcHasAlpha, float quality, bool colourRestrict,
                                                       bool alphaRestrict, float performance, void *out);
AL2O3_EXTERN_C void Image_CompressRichGel999BC7enc16(uint32_t const input[4 * 4], bool fast, bool perceptual,
                                                     void *out);

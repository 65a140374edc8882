// gic_api.cpp -- the C ABI of libgfx_imagecompress_amd.so.
//
// Two layers:
//   * gic_hip_* (include/gfx_imagecompress_amd/gic.h): batched, asynchronous
//     device entry points over images or float blocks resident in HBM.
//   * Image_Compress* (include/gfx_imagecompress/imagecompress.h): the
//     reference's host API (include/gfx_imagecompress/imagecompress.h:1-141),
//     implemented on top of gic_hip_* -- host image in, host image out, with
//     the reference's option defaults, destination-format choice, block-row
//     progress callback and NULL-on-failure contract.
// Every compression call runs the HIP kernels; there is no CPU fallback.

#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "../../include/gfx_imagecompress/imagecompress.h"
#include "../../include/gfx_imagecompress_amd/gic.h"
#include "gic_common.h"
#include "gic_pipeline.h"

namespace gic {
hipError_t launch_bc1_image(const Geometry &g, float thr, int steps, int force_alpha_one, int r3d, void *dst,
                            hipStream_t s);
hipError_t launch_bc45_image(const Geometry &g, int fmt, int channel, void *dst, hipStream_t s);
hipError_t launch_bc23_image(const Geometry &g, int fmt, int steps, int force_alpha_one, int r3d, void *dst,
                             hipStream_t s);
hipError_t launch_bc23_blocks(const float *blocks, uint32_t n, int fmt, int steps, int r3d, void *dst, hipStream_t s);
hipError_t launch_gather_f32(const Geometry &g, int kind, int force_alpha_one, uint32_t first, uint32_t n, float *out,
                             hipStream_t s);
hipError_t launch_bc45_rgba_blocks(const float *blocks, uint32_t n, int fmt, int channel, void *dst, hipStream_t s);
hipError_t launch_bcx_decode(const uint8_t *blocks, int fmt, uint32_t width, uint32_t height, uint32_t slices,
                             uint8_t *out, size_t row_pitch, hipStream_t s);
hipError_t launch_bc7_decode(const uint8_t *blocks, uint32_t width, uint32_t height, uint32_t slices, uint8_t *out,
                             size_t row_pitch, hipStream_t s);
hipError_t launch_bc1_blocks(const float *blocks, uint32_t n, float thr, int steps, int r3d, void *dst, hipStream_t s);
hipError_t launch_bc4_blocks(const float *blocks, uint32_t n, void *dst, hipStream_t s);
hipError_t launch_bc7_image(const Geometry &g, const gic_options &o, void *dst, double *err, hipStream_t s);
hipError_t launch_bc7_blocks(const float *blocks, uint32_t n, const gic_options &o, void *dst, double *err,
                             hipStream_t s);
hipError_t launch_bc7enc_image(const Geometry &g, const gic_options &o, void *dst, hipStream_t s);
hipError_t launch_bc7enc_blocks_u8(const uint32_t *blocks, uint32_t n, const gic_options &o, void *dst, hipStream_t s);
hipError_t launch_bc7enc_blocks_f32(const float *blocks, uint32_t n, const gic_options &o, void *dst, hipStream_t s);
hipError_t launch_bc6h_blocks(const float *blocks, uint32_t n, int is_signed, void *dst, double *err, hipStream_t s);
hipError_t launch_bc6h_decode(const uint8_t *blocks, uint32_t width, uint32_t height, uint32_t slices, int is_signed,
                              uint16_t *out, size_t row_pitch, hipStream_t s);
hipError_t launch_bc6h_image(const Geometry &g, int is_signed, int force_alpha_one, void *dst, double *err,
                             hipStream_t s);
hipError_t bc7_iter_cap(int cap, unsigned long long *hits, int reset);
hipError_t bc6h_iter_cap(int cap, unsigned long long *hits, int reset);
hipError_t bc7_nonterm(unsigned long long *n, int reset);
hipError_t bc6h_nonterm(unsigned long long *n, int reset);
void bc7_last_h4(uint32_t *rerun, uint32_t *nonterm);
void bc7_last_stages(uint32_t in[6], int *n);
}  // namespace gic

static bool is_bc6h(gic_format f) { return f == GIC_FMT_BC6H || f == GIC_FMT_BC6H_SF; }
// formats whose encoders report a per-block error (others write 0)
static bool has_error(gic_format f) { return f == GIC_FMT_BC7 || is_bc6h(f); }

static thread_local int t_last_hip_error = 0;

static int hip_fail(hipError_t e)
{
    t_last_hip_error = (int)e;
    fprintf(stderr, "gfx_imagecompress_amd: HIP error %d (%s)\n", (int)e, hipGetErrorString(e));
    return GIC_EHIP;
}

extern "C" int gic_last_hip_error(void) { return t_last_hip_error; }

extern "C" int gic_last_bc7_stages(uint32_t blocks_in[6], int *stages)
{
    if (!blocks_in || !stages) return GIC_EINVAL;
    gic::bc7_last_stages(blocks_in, stages);
    return GIC_OK;
}

extern "C" int gic_iter_cap_hits(unsigned long long *hits, int reset)
{
    if (!hits) return GIC_EINVAL;
    unsigned long long a = 0, b = 0;
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = gic::bc7_iter_cap(-1, &a, reset);
    if (e == hipSuccess) e = gic::bc6h_iter_cap(-1, &b, reset);
    if (e != hipSuccess) return hip_fail(e);
    *hits = a + b;
    return GIC_OK;
}

extern "C" int gic_set_iter_cap(int cap)
{
    if (cap < 0) cap = 4096;
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = gic::bc7_iter_cap(cap, nullptr, 0);
    if (e == hipSuccess) e = gic::bc6h_iter_cap(cap, nullptr, 0);
    return e == hipSuccess ? GIC_OK : hip_fail(e);
}

extern "C" int gic_nonterminating_loops(unsigned long long *loops, int reset)
{
    if (!loops) return GIC_EINVAL;
    unsigned long long a = 0, b = 0;
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = gic::bc7_nonterm(&a, reset);
    if (e == hipSuccess) e = gic::bc6h_nonterm(&b, reset);
    if (e != hipSuccess) return hip_fail(e);
    *loops = a + b;
    return GIC_OK;
}

extern "C" int gic_last_h4_report(uint32_t *rerun_blocks, uint32_t *nonterminating_loops)
{
    gic::bc7_last_h4(rerun_blocks, nonterminating_loops);
    return GIC_OK;
}

extern "C" const char *gic_version(void) { return "gfx_imagecompress_amd 0.1 (gfx950)"; }

extern "C" void gic_default_options(gic_options *o)
{
    if (!o) return;
    memset(o, 0, sizeof(*o));
    o->struct_size = sizeof(gic_options);
    o->bc1_alpha_threshold = 128 / 255.0f;   // amd_bc1_compressor.cpp:21-27,57
    o->refinement_steps = 1;                 // amd_bcx_helpers.cpp:23-31
    o->bc4_channel = 1;                      // amd_bc4_compressor.cpp:34
    o->bc7_mode_mask = 0xFF;
    o->colour_restrict = 1;                  // amd_bc7_compressor.cpp:58-65
    o->alpha_restrict = 1;
    o->bc7_quality = 1.0f;
    o->bc7_performance = 1.0f;
    o->bc7enc_perceptual = 1;                // richgel999_bc7enc16.cpp:13-19 ({perceptual, fast} = {true, false})
    o->bc7enc_uber_level = 4;                // :79 (BC7ENC16_MAX_UBER_LEVEL unless fast)
    o->bc7enc_max_partitions = 64;           // richgel999_bc7enc16.h:58
    o->bc7enc_least_squares = 1;
    o->bc7enc_filterbank = 1;
    o->bc7_mse_bound = 0.f;
}

extern "C" uint32_t gic_block_bytes(gic_format fmt)
{
    return (fmt == GIC_FMT_BC1 || fmt == GIC_FMT_BC4) ? 8u : 16u;
}

static int check_options(gic_format fmt, const gic_options &o)
{
    if (o.adaptive_weights) return GIC_EUNSUP;
    if (o.refinement_steps > 8) return GIC_EINVAL;
    if (fmt == GIC_FMT_BC4 && o.bc4_channel > 3) return GIC_EINVAL;
    if (o.bc7_performance != o.bc7_performance) return GIC_EINVAL;   // NaN (the reference clamps to [0, 1])
    if (o.bc7_shake_ranks > 8) return GIC_EINVAL;
    if (!(o.bc7_mse_bound >= 0.f) || o.bc7_mse_bound > 65025.f) return GIC_EINVAL;   // NaN, negative, > 255^2
    if (fmt == GIC_FMT_BC7ENC16 && (o.bc7enc_uber_level > 4 || o.bc7enc_max_partitions > 64)) return GIC_EINVAL;
    return GIC_OK;
}

static bool valid_fmt(gic_format f)
{
    return f == GIC_FMT_BC1 || f == GIC_FMT_BC2 || f == GIC_FMT_BC3 || f == GIC_FMT_BC4 || f == GIC_FMT_BC5 ||
           f == GIC_FMT_BC7 || f == GIC_FMT_BC7ENC16 || is_bc6h(f);
}

extern "C" int gic_hip_encode_rows(gic_format fmt, const uint8_t *d_src, uint32_t width, uint32_t height,
                                   uint32_t slices, uint32_t channels, size_t row_pitch, uint32_t first_block_row,
                                   uint32_t num_block_rows, const gic_options *opt, uint8_t *d_dst,
                                   double *d_block_err, void *stream)
{
    if (!valid_fmt(fmt) || !d_src || !d_dst || !width || !height || !slices || channels < 1 || channels > 4)
        return GIC_EINVAL;
    if (row_pitch < (size_t)width * channels) return GIC_EINVAL;
    const uint32_t by_count = (height + 3) / 4;
    if (first_block_row >= by_count || num_block_rows == 0 || first_block_row + num_block_rows > by_count)
        return GIC_EINVAL;
    gic_options o;
    gic_default_options(&o);
    if (opt) {
        if (opt->struct_size != sizeof(gic_options)) return GIC_EINVAL;
        o = *opt;
    }
    int rc = check_options(fmt, o);
    if (rc) return rc;
    const uint64_t total = (uint64_t)((width + 3) / 4) * num_block_rows * slices;
    if (total > 0xffffffffull) return GIC_EINVAL;
    gic::Geometry g;
    g.src = d_src;
    g.width = width;
    g.height = height;
    g.slices = slices;
    g.channels = channels;
    g.row_pitch = row_pitch;
    g.bx_count = (width + 3) / 4;
    g.row0 = first_block_row;
    g.nrows = num_block_rows;
    g.total = (uint32_t)total;
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipSuccess;
    if (d_block_err && !has_error(fmt)) {   // no encoder error but the AMD BC7 / BC6H ones
        e = hipMemsetAsync(d_block_err, 0, sizeof(double) * total, s);
        if (e != hipSuccess) return hip_fail(e);
    }
    switch (fmt) {
    case GIC_FMT_BC1:
        e = gic::launch_bc1_image(g, o.bc1_alpha_threshold, o.refinement_steps, o.force_alpha_one, o.b3d_refinement,
                                  d_dst, s);
        break;
    case GIC_FMT_BC2:
    case GIC_FMT_BC3:
        e = gic::launch_bc23_image(g, (int)fmt, o.refinement_steps, o.force_alpha_one, o.b3d_refinement, d_dst, s);
        break;
    case GIC_FMT_BC4:
    case GIC_FMT_BC5:
        e = gic::launch_bc45_image(g, (int)fmt, o.bc4_channel, d_dst, s);
        break;
    case GIC_FMT_BC7:
        e = gic::launch_bc7_image(g, o, d_dst, d_block_err, s);
        break;
    case GIC_FMT_BC7ENC16:
        e = gic::launch_bc7enc_image(g, o, d_dst, s);
        break;
    case GIC_FMT_BC6H:
    case GIC_FMT_BC6H_SF:
        e = gic::launch_bc6h_image(g, fmt == GIC_FMT_BC6H_SF, o.force_alpha_one, d_dst, d_block_err, s);
        break;
    default:
        break;
    }
    if (e != hipSuccess) return hip_fail(e);
    return GIC_OK;
}

extern "C" int gic_hip_encode_rows_src(gic_format fmt, gic_source src_type, const void *d_src, uint32_t width,
                                       uint32_t height, uint32_t slices, uint32_t channels, size_t row_pitch,
                                       uint32_t first_block_row, uint32_t num_block_rows, const gic_options *opt,
                                       uint8_t *d_dst, double *d_block_err, void *stream)
{
    if (src_type == GIC_SRC_UNORM8)
        return gic_hip_encode_rows(fmt, (const uint8_t *)d_src, width, height, slices, channels, row_pitch,
                                   first_block_row, num_block_rows, opt, d_dst, d_block_err, stream);
    if (src_type != GIC_SRC_SNORM8 && src_type != GIC_SRC_FLOAT32) return GIC_EINVAL;
    const size_t texel = (size_t)channels * (src_type == GIC_SRC_FLOAT32 ? 4 : 1);
    if (!valid_fmt(fmt) || !d_src || !d_dst || !width || !height || !slices || channels < 1 || channels > 4)
        return GIC_EINVAL;
    if (row_pitch < (size_t)width * texel) return GIC_EINVAL;
    const uint32_t by_count = (height + 3) / 4;
    if (first_block_row >= by_count || num_block_rows == 0 || first_block_row + num_block_rows > by_count)
        return GIC_EINVAL;
    gic_options o;
    gic_default_options(&o);
    if (opt) {
        if (opt->struct_size != sizeof(gic_options)) return GIC_EINVAL;
        o = *opt;
    }
    int rc = check_options(fmt, o);
    if (rc) return rc;
    const uint64_t total = (uint64_t)((width + 3) / 4) * num_block_rows * slices;
    if (total > 0xffffffffull) return GIC_EINVAL;
    gic::Geometry g;
    g.src = (const uint8_t *)d_src;
    g.width = width;
    g.height = height;
    g.slices = slices;
    g.channels = channels;
    g.row_pitch = row_pitch;
    g.bx_count = (width + 3) / 4;
    g.row0 = first_block_row;
    g.nrows = num_block_rows;
    g.total = (uint32_t)total;
    hipStream_t s = (hipStream_t)stream;
    const uint32_t chunk = total < (1u << 20) ? (uint32_t)total : (1u << 20);   // 256 MiB of float blocks
    float *tmp = nullptr;
    hipError_t e = hipMallocAsync((void **)&tmp, (size_t)chunk * 64 * sizeof(float), s);
    if (e != hipSuccess) return hip_fail(e);
    if (d_block_err && !has_error(fmt)) e = hipMemsetAsync(d_block_err, 0, sizeof(double) * total, s);
    const uint32_t bb = gic_block_bytes(fmt);
    const int force_alpha = o.force_alpha_one || channels < 4;
    for (uint32_t first = 0; e == hipSuccess && first < (uint32_t)total; first += chunk) {
        const uint32_t n = ((uint32_t)total - first) < chunk ? ((uint32_t)total - first) : chunk;
        e = gic::launch_gather_f32(g, src_type == GIC_SRC_SNORM8 ? 1 : 2, force_alpha, first, n, tmp, s);
        if (e != hipSuccess) break;
        uint8_t *out = d_dst + (size_t)first * bb;
        switch (fmt) {
        case GIC_FMT_BC1:
            e = gic::launch_bc1_blocks(tmp, n, o.bc1_alpha_threshold, o.refinement_steps, o.b3d_refinement, out, s);
            break;
        case GIC_FMT_BC2:
        case GIC_FMT_BC3:
            e = gic::launch_bc23_blocks(tmp, n, (int)fmt, o.refinement_steps, o.b3d_refinement, out, s);
            break;
        case GIC_FMT_BC4:
        case GIC_FMT_BC5:
            e = gic::launch_bc45_rgba_blocks(tmp, n, (int)fmt, o.bc4_channel, out, s);
            break;
        case GIC_FMT_BC7:
            e = gic::launch_bc7_blocks(tmp, n, o, out, d_block_err ? d_block_err + first : nullptr, s);
            break;
        case GIC_FMT_BC7ENC16:
            e = gic::launch_bc7enc_blocks_f32(tmp, n, o, out, s);
            break;
        case GIC_FMT_BC6H:
        case GIC_FMT_BC6H_SF:
            e = gic::launch_bc6h_blocks(tmp, n, fmt == GIC_FMT_BC6H_SF, out, d_block_err ? d_block_err + first : nullptr,
                                        s);
            break;
        default:
            break;
        }
    }
    const hipError_t ef = hipFreeAsync(tmp, s);
    if (e == hipSuccess) e = ef;
    if (e != hipSuccess) return hip_fail(e);
    return GIC_OK;
}

extern "C" int gic_hip_encode(gic_format fmt, const uint8_t *d_src, uint32_t width, uint32_t height,
                              uint32_t slices, uint32_t channels, size_t row_pitch, const gic_options *opt,
                              uint8_t *d_dst, double *d_block_err, void *stream)
{
    if (!height) return GIC_EINVAL;
    return gic_hip_encode_rows(fmt, d_src, width, height, slices, channels, row_pitch, 0, (height + 3) / 4, opt,
                               d_dst, d_block_err, stream);
}

extern "C" int gic_hip_encode_blocks_f32(gic_format fmt, const float *d_blocks, uint32_t n, const gic_options *opt,
                                         uint8_t *d_dst, double *d_block_err, void *stream)
{
    if (!d_blocks || !d_dst || !n) return GIC_EINVAL;
    if (fmt != GIC_FMT_BC1 && fmt != GIC_FMT_BC2 && fmt != GIC_FMT_BC3 && fmt != GIC_FMT_BC4 && fmt != GIC_FMT_BC7 &&
        fmt != GIC_FMT_BC7ENC16 && !is_bc6h(fmt))
        return GIC_EINVAL;
    gic_options o;
    gic_default_options(&o);
    if (opt) {
        if (opt->struct_size != sizeof(gic_options)) return GIC_EINVAL;
        o = *opt;
    }
    int rc = check_options(fmt, o);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipSuccess;
    // formats without an encoder error report 0 per block, as the row entries do
    if (d_block_err && !has_error(fmt)) e = hipMemsetAsync(d_block_err, 0, sizeof(double) * n, s);
    if (e != hipSuccess) return hip_fail(e);
    if (is_bc6h(fmt))
        e = gic::launch_bc6h_blocks(d_blocks, n, fmt == GIC_FMT_BC6H_SF, d_dst, d_block_err, s);
    else if (fmt == GIC_FMT_BC1)
        e = gic::launch_bc1_blocks(d_blocks, n, o.bc1_alpha_threshold, o.refinement_steps, o.b3d_refinement, d_dst, s);
    else if (fmt == GIC_FMT_BC4)
        e = gic::launch_bc4_blocks(d_blocks, n, d_dst, s);
    else if (fmt == GIC_FMT_BC2 || fmt == GIC_FMT_BC3)
        e = gic::launch_bc23_blocks(d_blocks, n, (int)fmt, o.refinement_steps, o.b3d_refinement, d_dst, s);
    else if (fmt == GIC_FMT_BC7ENC16)
        e = gic::launch_bc7enc_blocks_f32(d_blocks, n, o, d_dst, s);
    else
        e = gic::launch_bc7_blocks(d_blocks, n, o, d_dst, d_block_err, s);
    if (e != hipSuccess) return hip_fail(e);
    return GIC_OK;
}

extern "C" int gic_hip_encode_blocks_u8(gic_format fmt, const uint32_t *d_blocks, uint32_t n, const gic_options *opt,
                                        uint8_t *d_dst, void *stream)
{
    if (fmt != GIC_FMT_BC7ENC16 || !d_blocks || !d_dst || !n) return GIC_EINVAL;
    gic_options o;
    gic_default_options(&o);
    if (opt) {
        if (opt->struct_size != sizeof(gic_options)) return GIC_EINVAL;
        o = *opt;
    }
    int rc = check_options(fmt, o);
    if (rc) return rc;
    const hipError_t e = gic::launch_bc7enc_blocks_u8(d_blocks, n, o, d_dst, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e);
    return GIC_OK;
}

extern "C" int gic_hip_decode(gic_format fmt, const uint8_t *d_blocks, uint32_t width, uint32_t height,
                              uint32_t slices, uint8_t *d_rgba, size_t row_pitch, void *stream)
{
    if (!valid_fmt(fmt) || is_bc6h(fmt) || !d_blocks || !d_rgba || !width || !height || !slices) return GIC_EINVAL;
    if (row_pitch < (size_t)width * 4) return GIC_EINVAL;
    const hipError_t e = (fmt == GIC_FMT_BC7 || fmt == GIC_FMT_BC7ENC16)
                             ? gic::launch_bc7_decode(d_blocks, width, height, slices, d_rgba, row_pitch, (hipStream_t)stream)
                             : gic::launch_bcx_decode(d_blocks, (int)fmt, width, height, slices, d_rgba, row_pitch,
                                                      (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e);
    return GIC_OK;
}

extern "C" int gic_hip_decode_bc6h(gic_format fmt, const uint8_t *d_blocks, uint32_t width, uint32_t height,
                                   uint32_t slices, uint16_t *d_rgba16f, size_t row_pitch, void *stream)
{
    if (!is_bc6h(fmt) || !d_blocks || !d_rgba16f || !width || !height || !slices) return GIC_EINVAL;
    if (row_pitch < (size_t)width * 8 || (row_pitch & 1)) return GIC_EINVAL;
    const hipError_t e = gic::launch_bc6h_decode(d_blocks, width, height, slices, fmt == GIC_FMT_BC6H_SF, d_rgba16f,
                                                 row_pitch, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e);
    return GIC_OK;
}

// ------------------------------------------------------------------------
// Image model (stand-in for the un-vendored gfx_image, see gfx_image/image.h)
// ------------------------------------------------------------------------

extern "C" uint32_t TinyImageFormat_ChannelCount(TinyImageFormat f)
{
    switch (f) {
    case TinyImageFormat_R8_UNORM:
    case TinyImageFormat_R8_SNORM:
    case TinyImageFormat_DXBC4_UNORM:
    case TinyImageFormat_DXBC4_SNORM: return 1;
    case TinyImageFormat_R8G8_UNORM:
    case TinyImageFormat_R8G8_SNORM:
    case TinyImageFormat_DXBC5_UNORM:
    case TinyImageFormat_DXBC5_SNORM: return 2;
    case TinyImageFormat_R8G8B8_UNORM:
    case TinyImageFormat_R8G8B8_SRGB:
    case TinyImageFormat_DXBC1_RGB_UNORM:
    case TinyImageFormat_DXBC1_RGB_SRGB: return 3;
    case TinyImageFormat_R8G8B8A8_UNORM:
    case TinyImageFormat_R8G8B8A8_SRGB:
    case TinyImageFormat_R32G32B32A32_SFLOAT:
    case TinyImageFormat_DXBC1_RGBA_UNORM:
    case TinyImageFormat_DXBC1_RGBA_SRGB:
    case TinyImageFormat_DXBC2_UNORM:
    case TinyImageFormat_DXBC2_SRGB:
    case TinyImageFormat_DXBC3_UNORM:
    case TinyImageFormat_DXBC3_SRGB:
    case TinyImageFormat_DXBC7_UNORM:
    case TinyImageFormat_DXBC7_SRGB: return 4;
    case TinyImageFormat_DXBC6H_UFLOAT:
    case TinyImageFormat_DXBC6H_SFLOAT: return 3;
    default: return 0;
    }
}

extern "C" bool TinyImageFormat_IsSRGB(TinyImageFormat f)
{
    return f == TinyImageFormat_R8G8B8_SRGB || f == TinyImageFormat_R8G8B8A8_SRGB ||
           f == TinyImageFormat_DXBC1_RGB_SRGB || f == TinyImageFormat_DXBC1_RGBA_SRGB ||
           f == TinyImageFormat_DXBC2_SRGB || f == TinyImageFormat_DXBC3_SRGB || f == TinyImageFormat_DXBC7_SRGB;
}

extern "C" bool TinyImageFormat_IsSigned(TinyImageFormat f)
{
    return f == TinyImageFormat_R8_SNORM || f == TinyImageFormat_R8G8_SNORM || f == TinyImageFormat_DXBC4_SNORM ||
           f == TinyImageFormat_DXBC5_SNORM || f == TinyImageFormat_R32G32B32A32_SFLOAT ||
           f == TinyImageFormat_DXBC6H_SFLOAT;
}

extern "C" bool TinyImageFormat_IsFloat(TinyImageFormat f)
{
    return f == TinyImageFormat_R32G32B32A32_SFLOAT || f == TinyImageFormat_DXBC6H_UFLOAT ||
           f == TinyImageFormat_DXBC6H_SFLOAT;
}

extern "C" bool TinyImageFormat_IsCompressed(TinyImageFormat f) { return f >= TinyImageFormat_DXBC1_RGB_UNORM; }

extern "C" bool TinyImageFormat_IsNormalised(TinyImageFormat f)
{
    return f != TinyImageFormat_UNDEFINED && f != TinyImageFormat_R32G32B32A32_SFLOAT && f < TinyImageFormat_Count;
}

extern "C" uint32_t TinyImageFormat_BitSizeOfBlock(TinyImageFormat f)
{
    if (!TinyImageFormat_IsCompressed(f)) {
        if (f == TinyImageFormat_R32G32B32A32_SFLOAT) return 128;
        return 8 * TinyImageFormat_ChannelCount(f);
    }
    switch (f) {
    case TinyImageFormat_DXBC1_RGB_UNORM:
    case TinyImageFormat_DXBC1_RGB_SRGB:
    case TinyImageFormat_DXBC1_RGBA_UNORM:
    case TinyImageFormat_DXBC1_RGBA_SRGB:
    case TinyImageFormat_DXBC4_UNORM:
    case TinyImageFormat_DXBC4_SNORM: return 64;
    default: return 128;
    }
}

static uint64_t image_bytes(uint32_t w, uint32_t h, uint32_t d, uint32_t slices, TinyImageFormat f)
{
    if (TinyImageFormat_IsCompressed(f))
        return (uint64_t)((w + 3) / 4) * ((h + 3) / 4) * d * slices * (TinyImageFormat_BitSizeOfBlock(f) / 8);
    return (uint64_t)w * h * d * slices * (TinyImageFormat_BitSizeOfBlock(f) / 8);
}

extern "C" Image_ImageHeader const *Image_CreateNoClear(uint32_t w, uint32_t h, uint32_t d, uint32_t slices,
                                                        TinyImageFormat f)
{
    if (!w || !h || !d || !slices || f <= TinyImageFormat_UNDEFINED || f >= TinyImageFormat_Count) return nullptr;
    Image_ImageHeader *img = (Image_ImageHeader *)calloc(1, sizeof(Image_ImageHeader));
    if (!img) return nullptr;
    if (TinyImageFormat_IsCompressed(f)) {
        w = (w + 3) & ~3u;   // block formats pad to whole blocks
        h = (h + 3) & ~3u;
    }
    img->width = w;
    img->height = h;
    img->depth = d;
    img->slices = slices;
    img->format = f;
    img->dataSize = image_bytes(w, h, d, slices, f);
    img->data = gic::alloc_image_data(img->dataSize);
    if (!img->data) {
        free(img);
        return nullptr;
    }
    return img;
}

extern "C" Image_ImageHeader const *Image_Create(uint32_t w, uint32_t h, uint32_t d, uint32_t slices,
                                                 TinyImageFormat f)
{
    Image_ImageHeader const *img = Image_CreateNoClear(w, h, d, slices, f);
    if (img) memset(img->data, 0, img->dataSize);
    return img;
}

extern "C" void Image_Destroy(Image_ImageHeader const *img)
{
    if (!img) return;
    free(img->data);
    free((void *)img);
}

extern "C" void *Image_RawDataPtr(Image_ImageHeader const *img) { return img ? img->data : nullptr; }

// ------------------------------------------------------------------------
// Reference host API
// ------------------------------------------------------------------------

extern "C" void Image_CompressInit(void) {}
extern "C" void Image_CompressDeinit(void) {}

// Device scratch reused by the synchronous block-level and decode entry points of one thread.
struct DeviceScratch {
    void *src = nullptr, *dst = nullptr;
    size_t src_bytes = 0, dst_bytes = 0;
    hipStream_t stream = nullptr;
    ~DeviceScratch()
    {
        if (src) (void)hipFree(src);
        if (dst) (void)hipFree(dst);
        if (stream) (void)hipStreamDestroy(stream);
    }
    bool reserve(size_t sb, size_t db)
    {
        if (!stream && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return false;
        if (sb > src_bytes) {
            if (src) (void)hipFree(src);
            src = nullptr;
            src_bytes = 0;
            if (hipMalloc(&src, sb) != hipSuccess) return false;
            src_bytes = sb;
        }
        if (db > dst_bytes) {
            if (dst) (void)hipFree(dst);
            dst = nullptr;
            dst_bytes = 0;
            if (hipMalloc(&dst, db) != hipSuccess) return false;
            dst_bytes = db;
        }
        return true;
    }
};
static thread_local DeviceScratch t_scratch;

// The calling thread's lane (streams, events, device buffers) for host-image
// calls on one device; reused across calls, freed at thread exit.
struct ThreadLane {
    gic::LaneBuffers lb;
    ~ThreadLane() { lb.release(); }
};
static thread_local ThreadLane t_lane;
static thread_local gic_host_report t_host_report;

// GIC_DEVICES: a comma-separated device list for the image-level entry points.
// A list that cannot be parsed in full, or that names a device this process
// cannot see, is reported once and ignored (the call runs on one device).
static std::vector<int> env_devices()
{
    std::vector<int> out;
    const char *e = getenv("GIC_DEVICES");
    if (!e || !*e) return out;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) return {};
    bool bad = false;
    for (const char *p = e; *p && !bad;) {
        char *end = nullptr;
        const long v = strtol(p, &end, 10);
        if (end == p || v < 0 || v >= count || (*end && *end != ',')) {
            bad = true;
            break;
        }
        out.push_back((int)v);
        p = *end == ',' ? end + 1 : end;
    }
    if (bad) {
        static std::once_flag warned;
        std::call_once(warned, [e, count] {
            fprintf(stderr,
                    "gfx_imagecompress_amd: GIC_DEVICES=\"%s\" is not a comma-separated list of device "
                    "indices in [0, %d); running on the current device only\n", e, count);
        });
        return {};
    }
    return out;
}

// Host-image driver shared by the image-level wrappers: the block rows go
// through the upload / encode / download pipeline (gic_pipeline.cpp) on the
// current device, or on every device GIC_DEVICES lists; progress is reported
// per block row exactly as the reference loops do (amd_bc1_compressor.cpp:64-68),
// abort => NULL.
static Image_ImageHeader const *encode_host_image(Image_ImageHeader const *src, gic_format fmt, TinyImageFormat dst_fmt,
                                                  const gic_options &o, Image_CompressProgressFunc cb, void *user)
{
    t_host_report = gic_host_report{};
    if (!src || !src->data || src->depth > 1) return nullptr;
    const uint32_t ch = TinyImageFormat_ChannelCount(src->format);
    if (!ch || TinyImageFormat_IsCompressed(src->format)) return nullptr;
    // texel encoding (Image_GetPixelAtF, block_utils.cpp:24-26): the encoders
    // take any format the reference reads as floats
    const gic_source st = TinyImageFormat_IsFloat(src->format)    ? GIC_SRC_FLOAT32
                          : TinyImageFormat_IsSigned(src->format) ? GIC_SRC_SNORM8
                                                                  : GIC_SRC_UNORM8;
    const size_t texel_bytes = st == GIC_SRC_FLOAT32 ? 4 : 1;
    if (check_options(fmt, o) != GIC_OK) return nullptr;
    Image_ImageHeader const *dst = Image_CreateNoClear(src->width, src->height, 1, src->slices, dst_fmt);
    if (!dst) return nullptr;
    const size_t pitch = (size_t)src->width * ch * texel_bytes;
    const gic::EncodeArgs args{fmt, st, src->width, src->height, ch, pitch, &o};
    const std::vector<int> devs = env_devices();
    int rc;
    if (devs.size() > 1) {
        rc = gic::encode_host_devices(devs, args, (const uint8_t *)src->data, src->slices, (uint8_t *)dst->data, cb,
                                      user, &t_host_report);
    } else {
        int cur = 0;
        rc = hipGetDevice(&cur) == hipSuccess && t_lane.lb.lane.init(cur) == hipSuccess ? GIC_OK : GIC_EHIP;
        if (rc == GIC_OK)
            rc = gic::encode_host({&t_lane.lb}, args, (const uint8_t *)src->data, src->slices, (uint8_t *)dst->data,
                                  cb, user, &t_host_report);
        (void)hipSetDevice(cur);
    }
    if (rc != GIC_OK) {
        if (rc != GIC_EABORT)
            fprintf(stderr, "gfx_imagecompress_amd: GPU encode failed (%d, HIP error %d)\n", rc, gic_last_hip_error());
        Image_Destroy(dst);
        return nullptr;
    }
    return dst;
}

extern "C" int gic_last_host_report(gic_host_report *out)
{
    if (!out) return GIC_EINVAL;
    *out = t_host_report;
    return GIC_OK;
}

extern "C" Image_ImageHeader const *gic_compress_image(Image_ImageHeader const *src, gic_format fmt,
                                                       const gic_options *opt, bool (*progress)(void *, float),
                                                       void *user)
{
    if (!src || !valid_fmt(fmt)) return nullptr;
    gic_options o;
    gic_default_options(&o);
    if (opt) {
        if (opt->struct_size != sizeof(gic_options)) return nullptr;
        o = *opt;
    }
    const bool srgb = TinyImageFormat_IsSRGB(src->format), sgn = TinyImageFormat_IsSigned(src->format);
    const bool alpha = TinyImageFormat_ChannelCount(src->format) > 3;
    if (!alpha) o.force_alpha_one = 1;
    TinyImageFormat f = TinyImageFormat_UNDEFINED;
    switch (fmt) {
    case GIC_FMT_BC1:
        f = alpha ? (srgb ? TinyImageFormat_DXBC1_RGBA_SRGB : TinyImageFormat_DXBC1_RGBA_UNORM)
                  : (srgb ? TinyImageFormat_DXBC1_RGB_SRGB : TinyImageFormat_DXBC1_RGB_UNORM);
        break;
    case GIC_FMT_BC2: f = srgb ? TinyImageFormat_DXBC2_SRGB : TinyImageFormat_DXBC2_UNORM; break;
    case GIC_FMT_BC3: f = srgb ? TinyImageFormat_DXBC3_SRGB : TinyImageFormat_DXBC3_UNORM; break;
    case GIC_FMT_BC4: f = sgn ? TinyImageFormat_DXBC4_SNORM : TinyImageFormat_DXBC4_UNORM; break;
    case GIC_FMT_BC5: f = sgn ? TinyImageFormat_DXBC5_SNORM : TinyImageFormat_DXBC5_UNORM; break;
    case GIC_FMT_BC7:
    case GIC_FMT_BC7ENC16: f = srgb ? TinyImageFormat_DXBC7_SRGB : TinyImageFormat_DXBC7_UNORM; break;
    case GIC_FMT_BC6H: f = TinyImageFormat_DXBC6H_UFLOAT; break;
    case GIC_FMT_BC6H_SF: f = TinyImageFormat_DXBC6H_SFLOAT; break;
    default: return nullptr;
    }
    return encode_host_image(src, fmt, f, o, progress, user);
}

static Image_CompressAMDBackendOptions const kDefaultAmd = {false, false, 1, 0xFF};   // amd_bcx_helpers.cpp:23-31

extern "C" Image_ImageHeader const *Image_CompressAMDBC1(Image_ImageHeader const *src,
                                                         Image_CompressAMDBackendOptions const *amd,
                                                         Image_CompressBC1Options const *options,
                                                         Image_CompressProgressFunc cb, void *user)
{
    static Image_CompressBC1Options const kDefaultBc1 = {false, 128};   // amd_bc1_compressor.cpp:21-27
    if (!src) return nullptr;
    amd = amd ? amd : &kDefaultAmd;
    options = options ? options : &kDefaultBc1;
    const bool srgb = TinyImageFormat_IsSRGB(src->format);
    const bool dst_alpha = options->UseAlpha;
    // amd_bc1_compressor.cpp:33-35 (sRGB without alpha keeps the UNORM RGB format, as the reference does)
    TinyImageFormat f = srgb ? (dst_alpha ? TinyImageFormat_DXBC1_RGBA_SRGB : TinyImageFormat_DXBC1_RGB_UNORM)
                             : (dst_alpha ? TinyImageFormat_DXBC1_RGBA_UNORM : TinyImageFormat_DXBC1_RGB_UNORM);
    gic_options o;
    gic_default_options(&o);
    o.b3d_refinement = amd->b3DRefinement;
    o.adaptive_weights = amd->AdaptiveColourWeights;
    o.refinement_steps = amd->RefinementSteps;
    o.bc1_alpha_threshold = options->AlphaThreshold / 255.0f;
    o.force_alpha_one = TinyImageFormat_ChannelCount(src->format) > 3 ? 0 : 1;
    return encode_host_image(src, GIC_FMT_BC1, f, o, cb, user);
}

extern "C" Image_ImageHeader const *Image_CompressAMDBC4(Image_ImageHeader const *src, Image_CompressProgressFunc cb,
                                                         void *user)
{
    if (!src) return nullptr;
    TinyImageFormat f = TinyImageFormat_IsSigned(src->format) ? TinyImageFormat_DXBC4_SNORM : TinyImageFormat_DXBC4_UNORM;
    gic_options o;
    gic_default_options(&o);
    o.bc4_channel = 1;   // Q1: the reference reads green (amd_bc4_compressor.cpp:34-35)
    return encode_host_image(src, GIC_FMT_BC4, f, o, cb, user);
}

extern "C" Image_ImageHeader const *Image_CompressAMDBC5(Image_ImageHeader const *src, Image_CompressProgressFunc cb,
                                                         void *user)
{
    if (!src) return nullptr;
    TinyImageFormat f = TinyImageFormat_IsSigned(src->format) ? TinyImageFormat_DXBC5_SNORM : TinyImageFormat_DXBC5_UNORM;
    gic_options o;
    gic_default_options(&o);
    return encode_host_image(src, GIC_FMT_BC5, f, o, cb, user);
}

extern "C" Image_ImageHeader const *Image_CompressAMDBC7(Image_ImageHeader const *src,
                                                         Image_CompressAMDBackendOptions const *amd,
                                                         Image_CompressProgressFunc cb, void *user)
{
    if (!src) return nullptr;
    amd = amd ? amd : &kDefaultAmd;
    TinyImageFormat f = TinyImageFormat_IsSRGB(src->format) ? TinyImageFormat_DXBC7_SRGB : TinyImageFormat_DXBC7_UNORM;
    gic_options o;
    gic_default_options(&o);
    o.bc7_mode_mask = amd->ModeMask;   // amd_bc7_compressor.cpp:58-65
    o.force_alpha_one = TinyImageFormat_ChannelCount(src->format) > 3 ? 0 : 1;
    return encode_host_image(src, GIC_FMT_BC7, f, o, cb, user);
}

// BC2 / BC3 (amd_bc2_compressor.cpp:11-58, amd_bc3_compressor.cpp:11-58): sRGB
// sources give the sRGB destination; the colour half is the 4-colour fit of
// gic_bcx.hip encode_rgb4 (the reference's CompRGBBlock is undefined behaviour).
static Image_ImageHeader const *compress_bc23(Image_ImageHeader const *src, gic_format fmt,
                                              Image_CompressAMDBackendOptions const *amd, Image_CompressProgressFunc cb,
                                              void *user)
{
    if (!src) return nullptr;
    amd = amd ? amd : &kDefaultAmd;
    const bool srgb = TinyImageFormat_IsSRGB(src->format);
    const TinyImageFormat f = fmt == GIC_FMT_BC2 ? (srgb ? TinyImageFormat_DXBC2_SRGB : TinyImageFormat_DXBC2_UNORM)
                                                 : (srgb ? TinyImageFormat_DXBC3_SRGB : TinyImageFormat_DXBC3_UNORM);
    gic_options o;
    gic_default_options(&o);
    o.b3d_refinement = amd->b3DRefinement;
    o.adaptive_weights = amd->AdaptiveColourWeights;
    o.refinement_steps = amd->RefinementSteps;
    o.force_alpha_one = TinyImageFormat_ChannelCount(src->format) > 3 ? 0 : 1;
    return encode_host_image(src, fmt, f, o, cb, user);
}

extern "C" Image_ImageHeader const *Image_CompressAMDBC2(Image_ImageHeader const *src,
                                                         Image_CompressAMDBackendOptions const *amd,
                                                         Image_CompressProgressFunc cb, void *user)
{
    return compress_bc23(src, GIC_FMT_BC2, amd, cb, user);
}

extern "C" Image_ImageHeader const *Image_CompressAMDBC3(Image_ImageHeader const *src,
                                                         Image_CompressAMDBackendOptions const *amd,
                                                         Image_CompressProgressFunc cb, void *user)
{
    return compress_bc23(src, GIC_FMT_BC3, amd, cb, user);
}

// amd_bc6h_compressor.cpp:11-56: signed sources give DXBC6H_SFLOAT and the
// encoder's signed path, others DXBC6H_UFLOAT; quality 1.0; the ModeMask is
// passed to a constructor parameter that nothing reads, so it changes nothing.
extern "C" Image_ImageHeader const *Image_CompressAMDBC6H(Image_ImageHeader const *src,
                                                          Image_CompressAMDBackendOptions const *amd,
                                                          Image_CompressProgressFunc cb, void *user)
{
    if (!src) return nullptr;
    (void)amd;
    const bool sgn = TinyImageFormat_IsSigned(src->format);
    gic_options o;
    gic_default_options(&o);
    o.force_alpha_one = TinyImageFormat_ChannelCount(src->format) > 3 ? 0 : 1;
    return encode_host_image(src, sgn ? GIC_FMT_BC6H_SF : GIC_FMT_BC6H,
                             sgn ? TinyImageFormat_DXBC6H_SFLOAT : TinyImageFormat_DXBC6H_UFLOAT, o, cb, user);
}

// The bc7enc16 options of Image_CompressRichGel999BC7enc16 (richgel999_bc7enc16.cpp:73-89):
// perceptual or linear weights; fast = uber level 0, otherwise 4.
static void bc7enc_options(gic_options &o, bool fast, bool perceptual)
{
    o.bc7enc_perceptual = perceptual;
    o.bc7enc_uber_level = fast ? 0 : 4;
    o.bc7enc_max_partitions = 64;
    o.bc7enc_least_squares = 1;
    o.bc7enc_filterbank = 1;
}

// richgel999_bc7enc16.cpp:21-71: NULL options mean {perceptual = true, fast = false}
// (:13-19); sRGB sources give the sRGB destination; sources without alpha read alpha 1.
extern "C" Image_ImageHeader const *Image_CompressRichGel999BC7(Image_ImageHeader const *src,
                                                                Image_CompressRichGel999BackendOptions const *rich,
                                                                Image_CompressProgressFunc cb, void *user)
{
    static Image_CompressRichGel999BackendOptions const kDefaultRich = {true, false};
    if (!src) return nullptr;
    rich = rich ? rich : &kDefaultRich;
    TinyImageFormat f = TinyImageFormat_IsSRGB(src->format) ? TinyImageFormat_DXBC7_SRGB : TinyImageFormat_DXBC7_UNORM;
    gic_options o;
    gic_default_options(&o);
    bc7enc_options(o, rich->fast, rich->perceptual);
    o.force_alpha_one = TinyImageFormat_ChannelCount(src->format) > 3 ? 0 : 1;
    return encode_host_image(src, GIC_FMT_BC7ENC16, f, o, cb, user);
}

// imagecompress.cpp:20-50 (the reference's trailing Deinit is unreachable)
extern "C" Image_ImageHeader const *ImageCompress_Compress(Image_CompressType type, bool fast,
                                                            Image_ImageHeader const *src)
{
    Image_CompressInit();
    switch (type) {
    case Image_CT_None: return src;
    case Image_CT_DXBC1: return Image_CompressAMDBC1(src, nullptr, nullptr, nullptr, nullptr);
    case Image_CT_DXBC2: return Image_CompressAMDBC2(src, nullptr, nullptr, nullptr);
    case Image_CT_DXBC3: return Image_CompressAMDBC3(src, nullptr, nullptr, nullptr);
    case Image_CT_DXBC4: return Image_CompressAMDBC4(src, nullptr, nullptr);
    case Image_CT_DXBC5: return Image_CompressAMDBC5(src, nullptr, nullptr);
    case Image_CT_DXBC6H: return Image_CompressAMDBC6H(src, nullptr, nullptr, nullptr);
    case Image_CT_DXBC7:
        return fast ? Image_CompressRichGel999BC7(src, nullptr, nullptr, nullptr)
                    : Image_CompressAMDBC7(src, nullptr, nullptr, nullptr);
    default: return nullptr;
    }
}

// imagecompress.cpp:52-116
extern "C" Image_CompressType ImageCompress_PickCompressionType(Image_CompressPickFlags flags,
                                                                Image_ImageHeader const *src)
{
    if (!src) return Image_CT_None;
    if (TinyImageFormat_IsFloat(src->format)) {
        if ((flags & Image_CPF_AllowDXBC6and7) == 0) return Image_CT_None;
    } else if (!TinyImageFormat_IsNormalised(src->format)) {
        return Image_CT_None;
    }
    bool has_alpha = false;
    switch (TinyImageFormat_ChannelCount(src->format)) {
    case 1:
        if (flags & Image_CPF_AllowDXBC1to5) return Image_CT_DXBC4;
        break;
    case 2:
        if (flags & Image_CPF_AllowDXBC1to5) return Image_CT_DXBC5;
        break;
    case 3: break;
    case 4: has_alpha = true; break;
    }
    if (flags & Image_CPF_AllowDXBC6and7) return Image_CT_DXBC7;
    if (flags & Image_CPF_AllowASTC) return Image_CT_ASTC;
    if (has_alpha) {
        if (flags & Image_CPF_AllowDXBC1to5) return Image_CT_DXBC3;
        if (flags & Image_CPF_AllowETC) return Image_CT_None;
    } else {
        if (flags & Image_CPF_AllowDXBC1to5) return Image_CT_DXBC1;
        if (flags & Image_CPF_AllowETC) return Image_CT_None;
    }
    return Image_CT_None;
}

// ---- extensions: GPU decode of a compressed host image, DDS writer

static gic_format block_format_of(TinyImageFormat f)
{
    switch (f) {
    case TinyImageFormat_DXBC1_RGB_UNORM:
    case TinyImageFormat_DXBC1_RGB_SRGB:
    case TinyImageFormat_DXBC1_RGBA_UNORM:
    case TinyImageFormat_DXBC1_RGBA_SRGB: return GIC_FMT_BC1;
    case TinyImageFormat_DXBC2_UNORM:
    case TinyImageFormat_DXBC2_SRGB: return GIC_FMT_BC2;
    case TinyImageFormat_DXBC3_UNORM:
    case TinyImageFormat_DXBC3_SRGB: return GIC_FMT_BC3;
    case TinyImageFormat_DXBC4_UNORM:
    case TinyImageFormat_DXBC4_SNORM: return GIC_FMT_BC4;
    case TinyImageFormat_DXBC5_UNORM:
    case TinyImageFormat_DXBC5_SNORM: return GIC_FMT_BC5;
    case TinyImageFormat_DXBC7_UNORM:
    case TinyImageFormat_DXBC7_SRGB: return GIC_FMT_BC7;
    case TinyImageFormat_DXBC6H_UFLOAT: return GIC_FMT_BC6H;
    case TinyImageFormat_DXBC6H_SFLOAT: return GIC_FMT_BC6H_SF;
    default: return (gic_format)0;
    }
}

extern "C" Image_ImageHeader const *gic_decompress_image(Image_ImageHeader const *src)
{
    if (!src || !src->data) return nullptr;
    const gic_format fmt = block_format_of(src->format);
    if (!fmt) return nullptr;
    Image_ImageHeader const *dst =
        Image_CreateNoClear(src->width, src->height, 1, src->slices,
                            TinyImageFormat_IsSRGB(src->format) ? TinyImageFormat_R8G8B8A8_SRGB
                                                                : TinyImageFormat_R8G8B8A8_UNORM);
    if (!dst) return nullptr;
    const size_t blocks_bytes = (size_t)((src->width + 3) / 4) * ((src->height + 3) / 4) * src->slices *
                                gic_block_bytes(fmt);
    DeviceScratch &s = t_scratch;
    const bool ok = s.reserve(blocks_bytes, dst->dataSize) &&
                    hipMemcpyAsync(s.src, src->data, blocks_bytes, hipMemcpyHostToDevice, s.stream) == hipSuccess &&
                    gic_hip_decode(fmt, (const uint8_t *)s.src, src->width, src->height, src->slices,
                                   (uint8_t *)s.dst, (size_t)src->width * 4, s.stream) == GIC_OK &&
                    hipMemcpyAsync(dst->data, s.dst, dst->dataSize, hipMemcpyDeviceToHost, s.stream) == hipSuccess &&
                    hipStreamSynchronize(s.stream) == hipSuccess;
    if (!ok) {
        Image_Destroy(dst);
        return nullptr;
    }
    return dst;
}

// DDS: "DDS " + DDS_HEADER (124 bytes) [+ DDS_HEADER_DXT10 (20 bytes)] + data
extern "C" int gic_save_dds(Image_ImageHeader const *img, const char *path)
{
    if (!img || !img->data || !path) return GIC_EINVAL;
    const gic_format fmt = block_format_of(img->format);
    if (!fmt) return GIC_EINVAL;
    const bool srgb = TinyImageFormat_IsSRGB(img->format);
    const bool snorm = img->format == TinyImageFormat_DXBC4_SNORM || img->format == TinyImageFormat_DXBC5_SNORM;
    const bool dx10 = fmt == GIC_FMT_BC7 || is_bc6h(fmt) || srgb || snorm || img->slices > 1;
    // DXGI_FORMAT values of the DX10 header
    uint32_t dxgi = 0;
    switch (fmt) {
    case GIC_FMT_BC1: dxgi = srgb ? 72 : 71; break;
    case GIC_FMT_BC2: dxgi = srgb ? 75 : 74; break;
    case GIC_FMT_BC3: dxgi = srgb ? 78 : 77; break;
    case GIC_FMT_BC4: dxgi = snorm ? 81 : 80; break;
    case GIC_FMT_BC5: dxgi = snorm ? 84 : 83; break;
    case GIC_FMT_BC7:
    case GIC_FMT_BC7ENC16: dxgi = srgb ? 99 : 98; break;
    case GIC_FMT_BC6H: dxgi = 95; break;      // DXGI_FORMAT_BC6H_UF16
    case GIC_FMT_BC6H_SF: dxgi = 96; break;   // DXGI_FORMAT_BC6H_SF16
    }
    const uint32_t bb = gic_block_bytes(fmt);
    const uint32_t bx = (img->width + 3) / 4, by = (img->height + 3) / 4;
    uint32_t h[31];
    memset(h, 0, sizeof(h));
    h[0] = 124;                                   // dwSize
    h[1] = 0x1 | 0x2 | 0x4 | 0x1000 | 0x20000 | 0x80000;   // CAPS | HEIGHT | WIDTH | PIXELFORMAT | MIPMAPCOUNT | LINEARSIZE
    h[2] = img->height;
    h[3] = img->width;
    h[4] = bx * by * bb;                          // LINEARSIZE: bytes of the top-level image (one slice)
    h[6] = 1;                                     // mip levels
    h[18] = 32;                                   // DDS_PIXELFORMAT.dwSize
    h[19] = 0x4;                                  // DDPF_FOURCC
    auto fourcc = [](const char *c) {
        return (uint32_t)c[0] | ((uint32_t)c[1] << 8) | ((uint32_t)c[2] << 16) | ((uint32_t)c[3] << 24);
    };
    h[20] = dx10 ? fourcc("DX10")
                 : fourcc(fmt == GIC_FMT_BC1 ? "DXT1" : fmt == GIC_FMT_BC2 ? "DXT3" : fmt == GIC_FMT_BC3 ? "DXT5"
                                                     : fmt == GIC_FMT_BC4 ? "ATI1" : "ATI2");
    h[26] = 0x1000;                               // DDSCAPS_TEXTURE
    FILE *f = fopen(path, "wb");
    if (!f) return GIC_EHIP;
    bool ok = fwrite("DDS ", 1, 4, f) == 4 && fwrite(h, 4, 31, f) == 31;
    if (ok && dx10) {
        const uint32_t x[5] = {dxgi, 3 /* TEXTURE2D */, 0, img->slices, 0};
        ok = fwrite(x, 4, 5, f) == 5;
    }
    const size_t bytes = (size_t)bx * by * img->slices * bb;
    ok = ok && fwrite(img->data, 1, bytes, f) == bytes;
    ok = (fclose(f) == 0) && ok;
    return ok ? GIC_OK : GIC_EHIP;
}

// ---- block level: one-block GPU launches (prefer gic_hip_encode_blocks_f32 for batches)

static thread_local int t_block_status = GIC_OK;

extern "C" int gic_block_last_status(void) { return t_block_status; }

// One block's input and output in mapped pinned host memory: the kernels read
// the 64 floats and write the block words across PCIe themselves, so a call is
// a memcpy into the stage, the launches and one stream synchronisation -- no
// DMA copies in either direction (each pageable hipMemcpy was a staged copy of
// its own with a wait).
struct BlockStage {
    float *h_in = nullptr;
    uint8_t *h_out = nullptr;
    void *d_in = nullptr, *d_out = nullptr;
    ~BlockStage()
    {
        if (h_in) (void)hipHostFree(h_in);
        if (h_out) (void)hipHostFree(h_out);
    }
    bool ready()
    {
        if (d_in && d_out) return true;
        // fine-grained (coherent): the GPU never caches a previous call's block
        const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
        if (!h_in && hipHostMalloc((void **)&h_in, 64 * sizeof(float), fl) != hipSuccess) return false;
        if (!h_out && hipHostMalloc((void **)&h_out, 64, fl) != hipSuccess) return false;
        return hipHostGetDevicePointer(&d_in, h_in, 0) == hipSuccess &&
               hipHostGetDevicePointer(&d_out, h_out, 0) == hipSuccess;
    }
};
static thread_local BlockStage t_stage;

static bool encode_one_block(gic_format fmt, const float *in, size_t nfloats, const gic_options &o, void *out,
                             size_t out_bytes)
{
    DeviceScratch &s = t_scratch;
    BlockStage &b = t_stage;
    int st = GIC_OK;
    if (nfloats > 64 || out_bytes > 64 || !s.reserve(0, 0) || !b.ready()) st = GIC_EHIP;
    if (st == GIC_OK) {
        memcpy(b.h_in, in, nfloats * sizeof(float));
        st = gic_hip_encode_blocks_f32(fmt, (const float *)b.d_in, 1, &o, (uint8_t *)b.d_out, nullptr, s.stream);
    }
    if (st == GIC_OK && hipStreamSynchronize(s.stream) != hipSuccess) st = GIC_EHIP;
    if (st == GIC_OK) memcpy(out, b.h_out, out_bytes);
    t_block_status = st;
    if (st != GIC_OK) {
        fprintf(stderr, "gfx_imagecompress_amd: block encode failed (%d)\n", st);
        memset(out, 0, out_bytes);
    }
    return st == GIC_OK;
}

extern "C" void Image_CompressAMDBC1Block(float const input[64], bool adaptive, bool b3d, uint8_t steps,
                                          float alphaThreshold, void *out)
{
    gic_options o;
    gic_default_options(&o);
    o.adaptive_weights = adaptive;
    o.b3d_refinement = b3d;
    o.refinement_steps = steps;
    o.bc1_alpha_threshold = alphaThreshold;
    encode_one_block(GIC_FMT_BC1, input, 64, o, out, 8);
}

extern "C" void Image_CompressAMDAlphaSingleModeBlock(float const input[16], void *out)
{
    gic_options o;
    gic_default_options(&o);
    encode_one_block(GIC_FMT_BC4, input, 16, o, out, 8);
}

extern "C" void Image_CompressAMDMultiModeLDRBlock(float const input[64], uint8_t modeMask, bool srcHasAlpha,
                                                   float quality, bool colourRestrict, bool alphaRestrict,
                                                   float performance, void *out)
{
    (void)srcHasAlpha;   // unused by the reference encoder as well
    gic_options o;
    gic_default_options(&o);
    o.bc7_mode_mask = modeMask;
    o.bc7_quality = quality;
    o.bc7_performance = performance;
    o.colour_restrict = colourRestrict;
    o.alpha_restrict = alphaRestrict;
    encode_one_block(GIC_FMT_BC7, input, 64, o, out, 16);
}

// BC2/BC3 component blocks (amd_bcx_helpers.cpp:107-181): one BC2 block on the
// GPU built from the component, the requested half returned.
extern "C" void Image_CompressAMDRGBSingleModeBlock(float const rgb[48], bool adaptive, bool b3d, uint8_t steps,
                                                    void *out)
{
    float blk[64];
    for (int i = 0; i < 16; ++i) {
        blk[i * 4 + 0] = rgb[i * 3 + 0];
        blk[i * 4 + 1] = rgb[i * 3 + 1];
        blk[i * 4 + 2] = rgb[i * 3 + 2];
        blk[i * 4 + 3] = 1.0f;
    }
    gic_options o;
    gic_default_options(&o);
    o.adaptive_weights = adaptive;
    o.b3d_refinement = b3d;
    o.refinement_steps = steps;
    uint8_t b[16];
    if (encode_one_block(GIC_FMT_BC2, blk, 64, o, b, 16))
        memcpy(out, b + 8, 8);
    else
        memset(out, 0, 8);
}
extern "C" void Image_CompressAMDExplictAlphaSingleModeBlock(float const alpha[16], void *out)
{
    float blk[64];
    for (int i = 0; i < 16; ++i) {
        blk[i * 4 + 0] = blk[i * 4 + 1] = blk[i * 4 + 2] = 0.f;
        blk[i * 4 + 3] = alpha[i];
    }
    gic_options o;
    gic_default_options(&o);
    uint8_t b[16];
    if (encode_one_block(GIC_FMT_BC2, blk, 64, o, b, 16))
        memcpy(out, b, 8);
    else
        memset(out, 0, 8);
}
// richgel999_bc7enc16.cpp:73-97: one block of 16 packed RGBA8 texels
extern "C" void Image_CompressRichGel999BC7enc16(uint32_t const input[16], bool fast, bool perceptual, void *out)
{
    gic_options o;
    gic_default_options(&o);
    bc7enc_options(o, fast, perceptual);
    DeviceScratch &s = t_scratch;
    BlockStage &b = t_stage;
    bool ok = s.reserve(0, 0) && b.ready();
    if (ok) memcpy(b.h_in, input, 64);
    ok = ok &&
         gic_hip_encode_blocks_u8(GIC_FMT_BC7ENC16, (const uint32_t *)b.d_in, 1, &o, (uint8_t *)b.d_out, s.stream) ==
             GIC_OK &&
         hipStreamSynchronize(s.stream) == hipSuccess;
    if (ok) memcpy(out, b.h_out, 16);
    t_block_status = ok ? GIC_OK : GIC_EHIP;
    if (!ok) {
        fprintf(stderr, "gfx_imagecompress_amd: block encode failed on the GPU\n");
        memset(out, 0, 16);
    }
}

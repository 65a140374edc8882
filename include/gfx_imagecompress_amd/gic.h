/*
 * gic.h -- batched device entry points of the MI355X BCn compressor.
 *
 * C ABI only: plain pointers, sizes and a stream handle (a hipStream_t passed
 * as void*; NULL = the legacy default stream).  All pointers named d_* are
 * device (HBM) pointers.  These are the "new batched device entry" of
 * SURVEY.md section 8(b); the reference has no equivalent because its block
 * loop runs on the host (src/amd_bc1_compressor.cpp:44-70 and siblings).
 *
 * Return value: 0 on success, a negative number on error:
 *   GIC_EINVAL   bad argument (shape, pointer, option out of range)
 *   GIC_EUNSUP   option outside the implemented default-quality path
 *   GIC_EHIP     a HIP runtime call failed (see gic_last_hip_error())
 */
#ifndef GFX_IMAGECOMPRESS_AMD_GIC_H_
#define GFX_IMAGECOMPRESS_AMD_GIC_H_

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GIC_OK 0
#define GIC_EINVAL (-1)
#define GIC_EUNSUP (-2)
#define GIC_EHIP (-3)
#define GIC_EABORT (-4)   /* a progress callback asked to stop */

typedef enum gic_format {
    GIC_FMT_BC1 = 1, /* Image_CompressAMDBC1Block semantics (amd_bcx_helpers.cpp:51) */
    GIC_FMT_BC2 = 2, /* explicit 4-bit alpha (amd_bcx_helpers.cpp:107) + 4-colour RGB half */
    GIC_FMT_BC3 = 3, /* BC4-style alpha (:125) + 4-colour RGB half (amd_bc3_compressor.cpp:41-46) */
    GIC_FMT_BC4 = 4, /* Image_CompressAMDAlphaSingleModeBlock on one channel (:125) */
    GIC_FMT_BC5 = 5, /* two BC4 blocks, channel 0 then channel 1 (amd_bc5_compressor.cpp:35-41) */
    GIC_FMT_BC6H = 6, /* BC6HBlockEncoder::CompressBlock, unsigned half floats (amd_bc6h_body.cpp:1521,
                         Image_CompressAMDBC6H amd_bc6h_compressor.cpp:11 with an unsigned source) */
    GIC_FMT_BC7 = 7, /* BC7BlockEncoder::CompressBlock (amd_bc7_body.cpp:1289) */
    GIC_FMT_BC7ENC16 = 8, /* BC7 blocks (modes 1/6) by bc7enc16, the reference's fast BC7 encoder
                            (richgel999_bc7enc16.cpp:1517, Image_CompressRichGel999BC7 :21) */
    GIC_FMT_BC6H_SF = 9 /* BC6H with the encoder's m_isSigned set (a signed source such as
                           R32G32B32A32_SFLOAT, amd_bc6h_compressor.cpp:19-25) */
} gic_format;

/* Texel encodings of a source image (what Image_GetPixelAtF decodes). */
typedef enum gic_source {
    GIC_SRC_UNORM8 = 0, /* bytes, v / 255.0f (R8..R8G8B8A8 UNORM and sRGB) */
    GIC_SRC_SNORM8 = 1, /* signed bytes, max(v / 127.0f, -1.0f) (R8_SNORM, R8G8_SNORM) */
    GIC_SRC_FLOAT32 = 2 /* 32-bit floats as stored (R32G32B32A32_SFLOAT) */
} gic_source;

/* Options; gic_default_options() gives the reference defaults
 * (Image_CompressDefaultAmdOptions, amd_bcx_helpers.cpp:23-31; BC1 options,
 * amd_bc1_compressor.cpp:21-27; BC7 wrapper arguments, amd_bc7_compressor.cpp:58-65). */
typedef struct gic_options {
    uint32_t struct_size;        /* sizeof(gic_options) */
    float bc1_alpha_threshold;   /* 0..1; <= 0 disables punch-through (default 128/255) */
    uint8_t refinement_steps;    /* AMD RefinementSteps, 0..8 (default 1) */
    uint8_t b3d_refinement;      /* AMD b3DRefinement: Refine3D's joint 6-D endpoint jitter (BC1/BC2/BC3) */
    uint8_t adaptive_weights;    /* must be 0 (reference path is UB: block_utils.cpp:201-203) */
    uint8_t bc4_channel;         /* source channel for BC4 (reference reads 1: amd_bc4_compressor.cpp:34) */
    uint8_t bc7_mode_mask;       /* default 0xFF (0 means 0xCF, amd_bc7_body.hpp:103-106) */
    uint8_t colour_restrict;     /* default 1 */
    uint8_t alpha_restrict;      /* default 1 */
    uint8_t force_alpha_one;     /* 1: ignore source alpha (ReadNxNBlockF forceAlphaTo1) */
    float bc7_quality;           /* BC7BlockEncoder quality, clamped to [0,1] (default 1.0) */
    float bc7_performance;       /* BC7BlockEncoder performance, clamped to [0,1] (default 1.0); blocks whose
                                    range exceeds 255 * performance use the exhaustive optQuantTrace_d quantiser */
    uint32_t bc7_shake_ranks;    /* partitions shaken per single-index BC7 mode: 0 = the reference's
                                    count (8 at quality 1, bit-exact search); 1..8 caps it (pruned
                                    search, held to the per-block MSE tolerance) */
    /* bc7enc16 (GIC_FMT_BC7ENC16) settings, bc7enc16_compress_block_params
     * (richgel999_bc7enc16.h:17-36); defaults are the image API's
     * (Image_CompressDefaultRichGel99Options :13-19: perceptual, fast = false
     * -> uber level 4, Image_CompressRichGel999BC7enc16 :73-97) */
    uint8_t bc7enc_perceptual;      /* 1: YCbCr-weighted error, weights 128/64/16/32 (default 1) */
    uint8_t bc7enc_uber_level;      /* 0..4 (default 4; fast = true gives 0) */
    uint8_t bc7enc_max_partitions;  /* mode-1 partitions scanned, 0..64 (default 64) */
    uint8_t bc7enc_least_squares;   /* m_try_least_squares (default 1) */
    uint8_t bc7enc_filterbank;      /* m_mode1_partition_estimation_filterbank (default 1) */
    /* BC7 bounded exit (0 = off, the default): a cheap probe (modes 6, 3, then 1, mode 6 also on opaque blocks,
     * two partitions shaken) runs first and every block whose probe result
     * DECODES within this per-block MSE (RGBA, 0..255 units, mean over the 64
     * values) is final; only the other blocks run the full search.  With 0.5 --
     * the absolute slack of the BC7 contract MSE <= MSE_ref * (1 + 1e-3) + 0.5 --
     * every block meets the contract by construction.  Ignored below
     * quality 0.25, where the reference's own error-threshold exit is in force. */
    float bc7_mse_bound;
} gic_options;

void gic_default_options(gic_options *opt);

/* Bytes per 4x4 block of a format (8 or 16). */
uint32_t gic_block_bytes(gic_format fmt);

/* Encode a slice stack of 8-bit images resident in HBM.
 *   d_src: slices x height rows of row_pitch bytes, each texel `channels`
 *          bytes (1..4, R[G[B[A]]]), slice pitch = row_pitch * height.
 *   d_dst: blocks in row-major order per slice, slices stacked
 *          (ceil(w/4) * ceil(h/4) * slices * gic_block_bytes).
 *   d_block_err: optional (NULL) per-block error (BC7 / BC6H: the encoder's error, 0 for the others).
 * Partial edge blocks replicate the last row/column (block_utils.cpp:19-22).
 * The launch is asynchronous on `stream`. */
int gic_hip_encode(gic_format fmt, const uint8_t *d_src, uint32_t width, uint32_t height,
                   uint32_t slices, uint32_t channels, size_t row_pitch, const gic_options *opt,
                   uint8_t *d_dst, double *d_block_err, void *stream);

/* Same, restricted to block rows [first_block_row, first_block_row+num_block_rows)
 * of every slice; d_dst receives only those rows (contiguous per slice, slices
 * stacked).  This is the per-rank shard of the multi-GPU path. */
int gic_hip_encode_rows(gic_format fmt, const uint8_t *d_src, uint32_t width, uint32_t height,
                        uint32_t slices, uint32_t channels, size_t row_pitch,
                        uint32_t first_block_row, uint32_t num_block_rows, const gic_options *opt,
                        uint8_t *d_dst, double *d_block_err, void *stream);

/* gic_hip_encode_rows for any gic_source: UNORM8 runs the byte kernels
 * directly; SNORM8 / FLOAT32 texels are gathered into float blocks on the
 * device (stream-ordered scratch of <= 256 MiB) and encoded by the block-level
 * kernels (the reference's float block path: every format accepts any texels
 * Image_GetPixelAtF returns, block_utils.cpp:24-26).  row_pitch in bytes. */
int gic_hip_encode_rows_src(gic_format fmt, gic_source src_type, const void *d_src, uint32_t width,
                            uint32_t height, uint32_t slices, uint32_t channels, size_t row_pitch,
                            uint32_t first_block_row, uint32_t num_block_rows, const gic_options *opt,
                            uint8_t *d_dst, double *d_block_err, void *stream);

/* Multi-GPU encode from one host process (the split of the
 * reference's block loop, amd_bc1_compressor.cpp:44-70 / amd_bc7_compressor.cpp:
 * 48-77, across devices).  The block rows of every slice, numbered slice-major,
 * are cut into `ndev` contiguous ranges (the first rows % ndev one row longer);
 * device devices[i] uploads the source rows its range reads from the host image
 * `h_src` (slices x height rows of row_pitch bytes) and encodes them on its own
 * stream, every device from its own host thread; then ONE gather collects the
 * packed blocks at their reference-order offsets in `d_dst_root`, device
 * memory on devices[0] (ceil(w/4) * ceil(h/4) * slices * gic_block_bytes):
 * grouped ncclSend / ncclRecv over RCCL communicators (ncclCommInitAll over
 * the list, built once and kept until the list changes or gic_multi_release),
 * or peer copies when the list names a device twice or flags has
 * GIC_MULTI_PEER_COPY.  Returns after the gather completed; the calling
 * thread's current device is preserved.  Image_CompressAMD* use it when the
 * environment variable GIC_DEVICES lists more than one device (e.g. "0,1,2,3")
 * and no progress callback is given. */
#define GIC_MULTI_PEER_COPY 1u
typedef struct gic_multi_report {
    int ranks;               /* devices in the list */
    int rccl;                /* 1: the gather ran over RCCL, 0: peer copies */
    double encode_ms_max;    /* call start -> the slowest device's last encoded piece (host clock;
                                uploads and encodes pipelined per device) */
    double gather_ms;        /* the gather's exposed part: that moment -> the call's end (each
                                device sends as soon as its own encode is done) */
    uint64_t gathered_bytes; /* packed bytes received from the other devices */
} gic_multi_report;
int gic_encode_multi(gic_format fmt, gic_source src_type, const void *h_src, uint32_t width, uint32_t height,
                     uint32_t slices, uint32_t channels, size_t row_pitch, const gic_options *opt, int ndev,
                     const int *devices, uint8_t *d_dst_root, uint32_t flags);
/* the calling thread's last gic_encode_multi */
int gic_multi_last_report(gic_multi_report *out);
/* frees the device-list state (communicators, streams, buffers) */
int gic_multi_release(void);
/* the split: device i's first slice-major block row and row count (host only) */
int gic_multi_split(uint64_t rows_total, int ndev, int i, uint64_t *first, uint64_t *rows);

/* Host images (the Image_Compress* entry points and gic_compress_image).  The
 * reference's wrappers take a host image and return one (amd_bc1_compressor.cpp:
 * 36-70); here the block rows are cut into pieces (about 2^18 blocks, BC7 2^20)
 * and each device pipelines them: the upload of piece k+1 and the copy-out of
 * piece k-1 overlap the encode of piece k (gic_pipeline.cpp).  The upload mode
 * is the environment variable GIC_H2D: "pageable" (default: hipMemcpyAsync from
 * the caller's memory), "staged" (through a pinned ring) or "register"
 * (hipHostRegister of the caller's range for the call).  With GIC_DEVICES
 * listing several devices, every device pipelines its contiguous share of the
 * rows and downloads its blocks straight into the host image (no device
 * gather); a progress callback sees the reference's per-row sequence in the
 * reference's order in both cases, and returning true aborts (NULL). */
typedef struct gic_host_report {
    int devices;       /* devices the call ran on */
    int pieces;        /* pieces of block rows, over all devices */
    int h2d_mode;      /* 0 pageable, 1 staged, 2 register */
    double total_ms;   /* the whole call, host clock */
    double h2d_ms;     /* first upload start -> last upload end (HIP events; the slowest device) */
    double encode_ms;  /* first encode start -> last encode end */
    double d2h_ms;     /* first -> last copy of finished blocks into the host image (host clock; the
                          kernels write a host image's blocks straight into pinned host memory) */
} gic_host_report;
/* the calling thread's last host-image call */
int gic_last_host_report(gic_host_report *out);
/* Any format on a host image with explicit options (the Image_Compress*
 * wrappers fix the options the reference fixes; this entry takes them all, e.g.
 * the BC7 search options bc7_mse_bound / bc7_shake_ranks).  Destination format:
 * the wrappers' choice for the format (BC1: the RGBA variant for 4-channel
 * sources), sRGB for sRGB sources, SNORM BC4/BC5 for signed ones, BC6H signed for
 * GIC_FMT_BC6H_SF.  NULL on failure or abort; free with Image_Destroy. */
struct Image_ImageHeader;
struct Image_ImageHeader const *gic_compress_image(struct Image_ImageHeader const *src, gic_format fmt,
                                                   const gic_options *opt, bool (*progress)(void *user, float pct),
                                                   void *user);

/* Block-level batch: n blocks of 16 texels, float in [0,1].
 *   BC1/BC2/BC3/BC7: d_blocks holds n x 64 floats (RGBA per texel, texel-major).
 *   BC4:     d_blocks holds n x 16 floats.
 *   BC7ENC16: n x 64 floats, each texel to RGBA8 as saturate(v) * 255 + 0.5.
 *   BC6H / BC6H_SF: n x 64 floats (RGB used; any finite HDR value, converted to
 *     half floats as CompressBlock does, amd_bc6h_body.cpp:1539-1573).
 * This is the batched form of the reference's block API
 * (imagecompress.h:111-136). */
int gic_hip_encode_blocks_f32(gic_format fmt, const float *d_blocks, uint32_t n, const gic_options *opt,
                              uint8_t *d_dst, double *d_block_err, void *stream);

/* bc7enc16 at its block ABI (Image_CompressRichGel999BC7enc16,
 * richgel999_bc7enc16.cpp:73): n blocks of 16 packed RGBA8 texels
 * (R | G << 8 | B << 16 | A << 24, texel-major), 16-byte BC7 blocks out.
 * fmt must be GIC_FMT_BC7ENC16. */
int gic_hip_encode_blocks_u8(gic_format fmt, const uint32_t *d_blocks, uint32_t n, const gic_options *opt,
                             uint8_t *d_dst, void *stream);

/* Decode BCn blocks resident in HBM (row-major per slice, slices stacked, as
 * the encoders write them) to RGBA8: d_rgba receives slices x height rows of
 * row_pitch bytes, 4 bytes per texel (texels past the image edge are not
 * written).  Conventions (not part of the reference, which has no decoder):
 *   BC1/BC2/BC3 colour: 565 endpoints widened by bit replication, the 1/3 and
 *     2/3 points rounded to nearest; BC1 with c0 <= c1 is the 3-colour mode
 *     (midpoint rounded half up, index 3 = transparent black); BC2/BC3 colour
 *     blocks are always 4-colour;
 *   BC2 alpha: a4 * 17; BC3/BC4/BC5: the 8- or 6-level ramps rounded to
 *     nearest; BC4 -> (R, 0, 0, 255), BC5 -> (R, G, 0, 255);
 *   BC7: the BPTC format (weights round(64 i / (2^bits - 1)), reserved mode ->
 *     transparent black). */
int gic_hip_decode(gic_format fmt, const uint8_t *d_blocks, uint32_t width, uint32_t height, uint32_t slices,
                   uint8_t *d_rgba, size_t row_pitch, void *stream);

/* BC6H (GIC_FMT_BC6H / GIC_FMT_BC6H_SF) blocks to RGBA16F texels on the device:
 * 4 half-float bit patterns per texel (alpha 1.0), row_pitch >= width * 8 bytes,
 * decoded from the BC6H format description (not from the encoder's tables);
 * reserved modes decode to zero.  An extension: the reference has no decoder. */
int gic_hip_decode_bc6h(gic_format fmt, const uint8_t *d_blocks, uint32_t width, uint32_t height, uint32_t slices,
                        uint16_t *d_rgba16f, size_t row_pitch, void *stream);

/* Host image helpers (extensions; the reference has neither):
 *   gic_decompress_image: a BC1/BC2/BC3/BC4/BC5/BC7 image (as the
 *     Image_CompressAMD* functions return) decoded on the GPU to an RGBA8
 *     image (R8G8B8A8_SRGB for sRGB block formats), freed with Image_Destroy;
 *     NULL for other formats or on failure.
 *   gic_save_dds: writes a block-compressed image as a .dds file (legacy
 *     DXT1/DXT3/DXT5/ATI1/ATI2 FourCC header, DX10 extension header for BC7 and
 *     the sRGB variants) -- the SAVE_DDS step of the reference tests
 *     (tests/test_imagecompress.cpp:9-26, which use gfx_imageio).  Returns 0 or
 *     GIC_EINVAL / GIC_EHIP (I/O failure). */
struct Image_ImageHeader;
struct Image_ImageHeader const *gic_decompress_image(struct Image_ImageHeader const *src);
int gic_save_dds(struct Image_ImageHeader const *img, const char *path);

/* Last HIP error code recorded by this thread (0 if none). */
int gic_last_hip_error(void);

/* Status of this thread's last block-level call (Image_CompressAMD*Block,
 * Image_CompressRichGel999BC7enc16): GIC_OK, or the gic_* code of the failure.
 * Those entry points return void as in the reference (imagecompress.h:111-141);
 * a failed one writes a zero block, prints to stderr and sets this status. */
int gic_block_last_status(void);

/* Unbounded quantiser loops.  The reference's BC7 and BC6H
 * quantisers (optQuantAnD_d, amd_bc7_3dquant_vpc.cpp:1885-1986; optQuantAnD_f,
 * amd_hdr_encode.cpp:1427-1601) requantise in `do ... while (!done && try_two--)`
 * with a counter that is never reset: once it has run negative the loop runs
 * until the requantisation is stable, forever on a cycling state.  The loop's
 * state is the index vector alone, so a revisited state proves the reference
 * never returns.
 *  - BC7: the fast (register) quantisers stop a loop `cap` rounds past the
 *    counter's exhaustion (default 4096), count the stop and mark the block;
 *    every marked block is then encoded again through the general kernels,
 *    whose quantiser runs the reference's loop to its fixed point (a BC7 call
 *    returns with its device work complete for that reason).  The result is the
 *    reference's on every block where the reference returns; a loop proven
 *    cyclic stops and is counted as non-terminating.
 *  - BC6H: each loop stops at a proven cycle (non-terminating) or after `cap`
 *    rounds past the exhaustion within that loop (counted as a cap stop); the
 *    oracle (oracle/orc_bc6h.c) applies the same stops.  For BC6H both counters
 *    count loops per EXECUTED outer round: a proven outer-round cycle is
 *    fast-forwarded without running the skipped rounds' loops, so read the
 *    BC6H counts as a 0 / non-zero signal, not as the oracle's loop totals.
 *   gic_iter_cap_hits: cap stops since the last reset on the current device
 *     (synchronises the device); a BC7 stop means a re-run, not a wrong block;
 *   gic_set_iter_cap: the cap (< 0 restores 4096; a small cap is a test hook);
 *   gic_nonterminating_loops: loops proven cyclic since the last reset (the
 *     reference would never have returned on those blocks);
 *   gic_last_h4_report: this thread's last BC7 call -- blocks re-run after a
 *     cap stop, and loops proven cyclic during the call. */
int gic_iter_cap_hits(unsigned long long *hits, int reset);
int gic_set_iter_cap(int cap);
int gic_nonterminating_loops(unsigned long long *loops, int reset);
int gic_last_h4_report(uint32_t *rerun_blocks, uint32_t *nonterminating_loops);

/* Stages of the calling thread's last BC7 device call: *stages = 6 with the
 * bounded exit (bc7_mse_bound > 0: the direct mode-6 fit, the mode-6, mode-3,
 * mode-1 and mode-4 probes, then the full search; fewer if the mode mask drops
 * mode 6, 3, 1 or 4), 1 without; blocks_in[k] = blocks entering stage k (0 once
 * no block is left).  The bounded exit's probe-exit share is
 * 1 - blocks_in[stages - 1] / blocks_in[0]. */
int gic_last_bc7_stages(uint32_t blocks_in[6], int *stages);

/* Library version string. */
const char *gic_version(void);

#ifdef __cplusplus
}
#endif
#endif

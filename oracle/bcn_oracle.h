/*
 * bcn_oracle.h -- CPU restatement of the reference BCn block search.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * product path in gfx_imagecompress_amd/.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product never links it.
 *
 * Every function restates the algorithm of DeanoC/gfx_imagecompress (itself a
 * remix of AMD Compressonator) for the default-quality path, citing the
 * reference file:line it follows.  Parity pinning: see oracle/README.md and
 * tests/test_oracle.py (SURVEY.md section 8(c) fingerprints of the compiled
 * reference, recorded by the survey probe).
 */
#ifndef BCN_ORACLE_H_
#define BCN_ORACLE_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Image_CompressAMDBC1Block (amd_bcx_helpers.cpp:51-105).
 * in: 16 texels RGBA float [0,1]; alpha_threshold01 <= 0 disables alpha.
 * refinement_steps: AMD option RefinementSteps (default 1).  */
void orc_bc1_block(const float in[64], int refinement_steps,
                   float alpha_threshold01, uint8_t out[8]);

/* the same with the AMD b3DRefinement option (Refine3D, amd_bcx_body.cpp:808-932) */
void orc_bc1_block_ex(const float in[64], int refinement_steps, float alpha_threshold01, int b3d,
                      uint8_t out[8]);

/* Image_CompressAMDAlphaSingleModeBlock (amd_bcx_helpers.cpp:125-140). */
void orc_bc4_block(const float in[16], uint8_t out[8]);

/* BC2/BC3 halves: the 4-colour RGB block (alpha ignored; the reference's
 * CompRGBBlock is UB, see orc_bcx.c) and the explicit 4-bit alpha block. */
void orc_rgb4_block(const float in[64], int refinement_steps, int b3d, uint8_t out[8]);
void orc_explicit_alpha_block(const float in[16], uint8_t out[8]);

/* BC7BlockEncoder::CompressBlock (amd_bc7_body.cpp:1289-1465) with the
 * encoder constructed as in Image_CompressAMDMultiModeLDRBlock
 * (amd_bc7_compressor.cpp:11-23).  Returns the encoder's block error. */
double orc_bc7_block(const float in[64], uint8_t mode_mask, int src_has_alpha,
                     float quality, int colour_restrict, int alpha_restrict,
                     float performance, uint8_t out[16]);

/* orc_bc7_block with the GPU's optional shake-rank cap (gic_options.bc7_shake_ranks;
 * 0 = the reference). */
double orc_bc7_block_ex(const float in[64], uint8_t mode_mask, int src_has_alpha,
                        float quality, int colour_restrict, int alpha_restrict,
                        float performance, int shake_ranks, uint8_t out[16]);

/* Image-level drivers over an 8-bit source (the reference's block loops in
 * amd_bc{1,4,5,7}_compressor.cpp with ReadNxNBlockF edge clamping,
 * block_utils.cpp:7-41, and UNORM8 -> float as v/255.0f).
 * src: rows of width*channels bytes, slices stacked; dst: row-major blocks.
 * fmt: 1 = BC1, 2 = BC2, 3 = BC3, 4 = BC4, 5 = BC5, 7 = BC7.  channels in {1,2,3,4}.
 * bc4_channel selects the source channel for BC4 (reference uses 1).
 * first_row/num_rows restrict to a block-row range (per slice); rows <0 = all.
 * threads: 0/1 = calling thread, N = a pool of N pthreads over block rows. */
int orc_encode_image(int fmt, const uint8_t *src, uint32_t width, uint32_t height,
                     uint32_t slices, uint32_t channels, int bc4_channel,
                     int32_t first_row, int32_t num_rows, int threads,
                     uint8_t *dst, double *block_err);

/* The BC7 block loop with the encoder's quality and ModeMask exposed (the
 * reference's image API fixes quality 1.0, amd_bc7_compressor.cpp:58-65; the
 * block API Image_CompressAMDMultiModeLDRBlock takes both). */
int orc_encode_image_bc7(const uint8_t *src, uint32_t width, uint32_t height, uint32_t slices, uint32_t channels,
                         int32_t first_row, int32_t num_rows, int threads, float quality, uint8_t mode_mask,
                         uint8_t *dst, double *block_err);
int orc_encode_image_bc7_ex(const uint8_t *src, uint32_t width, uint32_t height, uint32_t slices, uint32_t channels,
                            int32_t first_row, int32_t num_rows, int threads, float quality, uint8_t mode_mask,
                            int shake_ranks, uint8_t *dst, double *block_err);

/* bc7enc16, the reference's fast BC7 encoder (richgel999_bc7enc16.cpp):
 * Image_CompressRichGel999BC7enc16 on one packed RGBA8 block (:73-97) and the
 * Image_CompressRichGel999BC7 block loop over an 8-bit image (:21-71). */
void orc_bc7enc_block(const uint8_t rgba[64], int fast, int perceptual, uint8_t out[16]);
int orc_encode_image_bc7enc(const uint8_t *src, uint32_t width, uint32_t height, uint32_t slices, uint32_t channels,
                            int fast, int perceptual, uint8_t *dst);
/* the same through the image driver's block-row range and thread pool */
int orc_encode_image_bc7enc_rows(const uint8_t *src, uint32_t width, uint32_t height, uint32_t slices,
                                 uint32_t channels, int32_t first_row, int32_t num_rows, int threads, int fast,
                                 int perceptual, uint8_t *dst);

/* the BC7 block loop with the encoder's performance as well (optQuantTrace_d below 1) */
int orc_encode_image_bc7_perf(const uint8_t *src, uint32_t width, uint32_t height, uint32_t slices, uint32_t channels,
                              int32_t first_row, int32_t num_rows, int threads, float quality, uint8_t mode_mask,
                              float performance, uint8_t *dst, double *block_err);

/* BC6HBlockEncoder::CompressBlock (amd_bc6h_body.cpp:1521-1652) as
 * Image_CompressAMDBC6H constructs it (quality 1.0, amd_bc6h_compressor.cpp:28):
 * in = 16 RGBA float texels (alpha ignored); returns the encoder's error.
 * Parity-unpinned: Math_Float2Half is taken as IEEE binary16 RNE (orc_bc6h.c). */
float orc_bc6h_block(const float in[64], int is_signed, uint8_t out[16]);
int orc_encode_bc6h_blocks(const float *blocks, int n, int is_signed, int threads, uint8_t *out, float *err);
/* H4 stops of optQuantAnD_f's requantisation loop: the per-loop cap (rounds past
 * try_two's exhaustion, < 0 = 4096) and the cumulative stop counts (proven
 * cycles, cap hits) */
void orc_bc6h_set_cap(int cap);
void orc_bc6h_h4_counts(unsigned long long *nonterm, unsigned long long *capped);
/* test hooks: FindBestPattern of one pattern (-1 = one region), the half
 * conversion, the BPTC anchors, eigenVector_d's squaring count */
float orc_bc6h_pattern(const float in[64], int is_signed, int shape, float fep[12], int idx[32], int cnt[2]);
uint16_t orc_float_to_half(float f);
int orc_bc6h_anchor(int shape, int *pos);
int orc_bc6h_ev_p(void);

/* bounded-exit probe model: mode 6 starts its shake from the quantiser's
 * first projection (thread-local switch; not the reference) */
void orc_bc7_set_probe_init(int on);
/* bounded-exit stage 0 model (gic_bc7.hip k_fit6): the direct mode-6 fit of one
 * block; returns its palette's squared error */
double orc_bc7_fit6(const float in[64], uint8_t out[16]);

/* helpers exposed for unit tests */
void orc_load_block_rgba8(const uint8_t *src, uint32_t width, uint32_t height,
                          uint32_t channels, uint32_t bx, uint32_t by,
                          int force_alpha_one, float out[64]);
uint64_t orc_fnv1a64(const uint8_t *p, size_t n);
/* BC7 reference-style ramp value used by the shakers (amd_shake.cpp:283-286) */
int orc_bc7_shake_ramp(int clog, int bits, int p1, int p2, int i);
/* optQuantAnD_d on caller data, data4 = n x 4 doubles (test hook) */
double orc_bc7_opt_quant(const double *data4, int n, int ncl, int *index, int dim);
/* optQuantTrace_d on caller data (n <= 16), and the traceBuilder tables (test hooks) */
double orc_bc7_opt_quant_trace(const double *data4, int n, int ncl, int *index, int dim);
int orc_bc7_trace_len(int nc, int ne);
void orc_bc7_trace_step(int nc, int ne, int i, int *k, int *code, double *d);
/* decode one BC7 block to RGBA8 (for tolerance checks) */
void orc_bc7_decode(const uint8_t blk[16], uint8_t rgba[64]);
void orc_bc7_decode_n(const uint8_t *blk, size_t n, uint8_t *rgba);

#ifdef __cplusplus
}
#endif
#endif

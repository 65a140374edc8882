/*
 * orc_image.c -- image-level drivers for the CPU restatement.
 *
 * TEST INFRASTRUCTURE ONLY (see bcn_oracle.h).  Restates the block loops of
 * src/amd_bc{1,4,5,7}_compressor.cpp (raster order over slices, block rows,
 * block columns) and ReadNxNBlockF / ReadNxNSingleBlockF edge clamping
 * (src/block_utils.cpp:7-41, :116-144).  The UNORM8 -> float conversion
 * (Image_GetPixelAtF in the un-vendored gfx_image) is restated as v/255.0f.
 * A pthread pool over block rows (BC7: pieces of 16 blocks of a row) provides the
 * multi-core CPU baseline.
 */
#include "bcn_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

uint64_t orc_fnv1a64(const uint8_t *p, size_t n)
{
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < n; ++i) {
        h ^= p[i];
        h *= 0x100000001b3ull;
    }
    return h;
}

static float unorm8(uint8_t v) { return (float)v / 255.0f; }

/* ReadNxNBlockF, block_utils.cpp:7-41: x/y beyond the image clamp to the
 * last column/row.  Missing channels read as 0 (alpha as 1). */
void orc_load_block_rgba8(const uint8_t *src, uint32_t width, uint32_t height, uint32_t channels,
                          uint32_t bx, uint32_t by, int force_alpha_one, float out[64])
{
    for (uint32_t y = 0; y < 4; ++y) {
        uint32_t sy = by * 4 + y;
        if (sy >= height) sy = height - 1;
        for (uint32_t x = 0; x < 4; ++x) {
            uint32_t sx = bx * 4 + x;
            if (sx >= width) sx = width - 1;
            const uint8_t *p = src + ((size_t)sy * width + sx) * channels;
            float *o = out + (y * 4 + x) * 4;
            o[0] = unorm8(p[0]);
            o[1] = channels > 1 ? unorm8(p[1]) : 0.f;
            o[2] = channels > 2 ? unorm8(p[2]) : 0.f;
            o[3] = channels > 3 ? unorm8(p[3]) : 1.f;
            if (force_alpha_one) o[3] = 1.0f;
        }
    }
}

typedef struct {
    int fmt;
    const uint8_t *src;
    uint32_t width, height, slices, channels;
    int bc4_channel;
    uint32_t row0, nrows, bx_count, by_count;
    uint8_t *dst;
    double *err;
    float bc7_quality;   /* BC7BlockEncoder quality (image API: 1.0) */
    uint8_t bc7_mask;    /* BC7 ModeMask (image API default 0xFF) */
    int bc7_ranks;       /* shake-rank cap (0 = reference) */
    int enc_fast, enc_perceptual;   /* bc7enc16 (fmt 8) settings */
    float bc7_perf;      /* BC7BlockEncoder performance (image API: 1.0) */
    int next;            /* next job ((slice*nrows + row)*row_jobs + column piece) */
    int njobs;
    uint32_t row_jobs;   /* jobs per block row: 1, or pieces of kBc7Piece blocks for BC7 */
    pthread_mutex_t lock;
} job_t;

enum { kBc7Piece = 16 };   /* BC7 job size in blocks */

static size_t block_bytes(int fmt) { return (fmt == 1 || fmt == 4) ? 8 : 16; }
static int g_enc_fast, g_enc_perceptual;   /* set by orc_encode_image_bc7enc_rows before the pool runs */
static __thread float t_bc7_perf = 1.0f;   /* set by orc_encode_image_bc7_perf for its own call */

static void encode_row(job_t *j, uint32_t slice, uint32_t brow, uint32_t bx0, uint32_t bx1)
{
    const size_t slice_px = (size_t)j->width * j->height * j->channels;
    const uint8_t *img = j->src + slice_px * slice;
    const size_t bb = block_bytes(j->fmt);
    const int has_alpha = j->channels > 3;
    /* output is the shard's own contiguous region: rows [row0,row0+nrows) of every slice */
    const size_t out_row = ((size_t)slice * j->nrows + (brow - j->row0)) * j->bx_count;
    for (uint32_t bx = bx0; bx < bx1; ++bx) {
        float blk[64], ch[16];
        uint8_t *o = j->dst + (out_row + bx) * bb;
        double e = 0.0;
        orc_load_block_rgba8(img, j->width, j->height, j->channels, bx, brow, !has_alpha, blk);
        switch (j->fmt) {
        case 1:
            /* Image_CompressAMDBC1 defaults: steps 1, threshold 128/255 */
            orc_bc1_block(blk, 1, 128 / 255.0f, o);
            break;
        case 2:
        case 3:
            /* amd_bc{2,3}_compressor.cpp:36-50: alpha half, then the colour half */
            for (int i = 0; i < 16; ++i) ch[i] = blk[i * 4 + 3];
            if (j->fmt == 3)
                orc_bc4_block(ch, o);
            else
                orc_explicit_alpha_block(ch, o);
            orc_rgb4_block(blk, 1, 0, o + 8);
            break;
        case 4:
            for (int i = 0; i < 16; ++i) ch[i] = blk[i * 4 + j->bc4_channel];
            orc_bc4_block(ch, o);
            break;
        case 5:
            for (int i = 0; i < 16; ++i) ch[i] = blk[i * 4 + 0];
            orc_bc4_block(ch, o);
            for (int i = 0; i < 16; ++i) ch[i] = blk[i * 4 + 1];
            orc_bc4_block(ch, o + 8);
            break;
        case 7:
            /* Image_CompressAMDBC7 (amd_bc7_compressor.cpp:58-65) */
            e = orc_bc7_block_ex(blk, j->bc7_mask, has_alpha, j->bc7_quality, 1, 1, j->bc7_perf, j->bc7_ranks, o);
            break;
        case 8: {
            /* Image_CompressRichGel999BC7 (richgel999_bc7enc16.cpp:50-57): the float
             * block back to RGBA8 -- the identity on v / 255.0f */
            uint8_t px[64];
            for (int i = 0; i < 64; ++i) {
                const float v = blk[i] < 0.f ? 0.f : (blk[i] > 1.f ? 1.f : blk[i]);
                px[i] = (uint8_t)(v * 255.0f + 0.5f);
            }
            orc_bc7enc_block(px, j->enc_fast, j->enc_perceptual, o);
            break;
        }
        }
        if (j->err) j->err[out_row + bx] = e;
    }
}

static void *worker(void *arg)
{
    job_t *j = (job_t *)arg;
    for (;;) {
        pthread_mutex_lock(&j->lock);
        int k = j->next++;
        pthread_mutex_unlock(&j->lock);
        if (k >= j->njobs) break;
        const uint32_t piece = (uint32_t)k % j->row_jobs, rk = (uint32_t)k / j->row_jobs;
        const uint32_t w = (j->bx_count + j->row_jobs - 1) / j->row_jobs;
        const uint32_t bx0 = piece * w, bx1 = bx0 + w < j->bx_count ? bx0 + w : j->bx_count;
        if (bx0 < bx1) encode_row(j, rk / j->nrows, j->row0 + rk % j->nrows, bx0, bx1);
    }
    return NULL;
}

static int encode_image(int fmt, const uint8_t *src, uint32_t width, uint32_t height, uint32_t slices,
                        uint32_t channels, int bc4_channel, int32_t first_row, int32_t num_rows, int threads,
                        float bc7_quality, uint8_t bc7_mask, int bc7_ranks, uint8_t *dst, double *block_err)
{
    if (!src || !dst || !width || !height || !slices || channels < 1 || channels > 4) return -1;
    if (fmt < 1 || fmt > 8 || fmt == 6) return -1;
    job_t j;
    memset(&j, 0, sizeof(j));
    j.fmt = fmt;
    j.src = src;
    j.width = width;
    j.height = height;
    j.slices = slices;
    j.channels = channels;
    j.bc4_channel = bc4_channel;
    j.bc7_quality = bc7_quality;
    j.bc7_mask = bc7_mask;
    j.bc7_ranks = bc7_ranks;
    j.enc_fast = g_enc_fast;
    j.bc7_perf = t_bc7_perf;
    j.enc_perceptual = g_enc_perceptual;
    j.bx_count = (width + 3) / 4;
    j.by_count = (height + 3) / 4;
    j.row0 = first_row < 0 ? 0 : (uint32_t)first_row;
    j.nrows = num_rows < 0 ? j.by_count - j.row0 : (uint32_t)num_rows;
    if (j.row0 + j.nrows > j.by_count) return -1;
    j.dst = dst;
    j.err = block_err;
    /* BC7 costs ~10 ms per block on one core: a block row is split into pieces of
     * kBc7Piece blocks so that a sample of a few rows still keeps every thread busy */
    j.row_jobs = fmt == 7 ? (j.bx_count + kBc7Piece - 1) / kBc7Piece : 1;
    j.njobs = (int)(j.nrows * slices * j.row_jobs);
    pthread_mutex_init(&j.lock, NULL);
    if (threads <= 1) {
        worker(&j);
    } else {
        pthread_t *t = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
        for (int i = 0; i < threads; ++i) pthread_create(&t[i], NULL, worker, &j);
        for (int i = 0; i < threads; ++i) pthread_join(t[i], NULL);
        free(t);
    }
    pthread_mutex_destroy(&j.lock);
    return 0;
}

int orc_encode_image(int fmt, const uint8_t *src, uint32_t width, uint32_t height, uint32_t slices,
                     uint32_t channels, int bc4_channel, int32_t first_row, int32_t num_rows,
                     int threads, uint8_t *dst, double *block_err)
{
    return encode_image(fmt, src, width, height, slices, channels, bc4_channel, first_row, num_rows, threads, 1.0f,
                        0xFF, 0, dst, block_err);
}

int orc_encode_image_bc7(const uint8_t *src, uint32_t width, uint32_t height, uint32_t slices, uint32_t channels,
                         int32_t first_row, int32_t num_rows, int threads, float quality, uint8_t mode_mask,
                         uint8_t *dst, double *block_err)
{
    return encode_image(7, src, width, height, slices, channels, 0, first_row, num_rows, threads, quality,
                        mode_mask, 0, dst, block_err);
}

int orc_encode_image_bc7_ex(const uint8_t *src, uint32_t width, uint32_t height, uint32_t slices, uint32_t channels,
                            int32_t first_row, int32_t num_rows, int threads, float quality, uint8_t mode_mask,
                            int shake_ranks, uint8_t *dst, double *block_err)
{
    return encode_image(7, src, width, height, slices, channels, 0, first_row, num_rows, threads, quality,
                        mode_mask, shake_ranks, dst, block_err);
}

int orc_encode_image_bc7enc_rows(const uint8_t *src, uint32_t width, uint32_t height, uint32_t slices,
                                 uint32_t channels, int32_t first_row, int32_t num_rows, int threads, int fast,
                                 int perceptual, uint8_t *dst)
{
    g_enc_fast = fast;
    g_enc_perceptual = perceptual;
    return encode_image(8, src, width, height, slices, channels, 0, first_row, num_rows, threads, 1.0f, 0xFF, 0,
                        dst, NULL);
}

int orc_encode_image_bc7_perf(const uint8_t *src, uint32_t width, uint32_t height, uint32_t slices, uint32_t channels,
                              int32_t first_row, int32_t num_rows, int threads, float quality, uint8_t mode_mask,
                              float performance, uint8_t *dst, double *block_err)
{
    t_bc7_perf = performance;
    const int rc = encode_image(7, src, width, height, slices, channels, 0, first_row, num_rows, threads, quality,
                                mode_mask, 0, dst, block_err);
    t_bc7_perf = 1.0f;
    return rc;
}

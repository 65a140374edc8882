/* Lane utilisation of the BC1 kernel's data-dependent axis loop
 * (CompressRGBBlockX for(;;), amd_bcx_body.cpp:1034-1182; gic_bcx.hip
 * fit_endpoints), measured with the oracle's iteration counters: one lane per
 * block, 64 consecutive blocks of a block row per wavefront, so a wave runs
 * the 3-colour loop max-over-lanes times and the 4-colour loop (skipped when
 * the 3-colour error is 0) likewise.
 *   gcc -O2 -DORC_STATS -ffp-contract=off -I oracle tools/bc1_iter_study.c oracle/orc_*.c -lm -lpthread -o /tmp/bc1s
 *   /tmp/bc1s <rows> [noise]   (rows of the 8192^2 G1 texture, every 2048/rows-th row) */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include "bcn_oracle.h"

extern __thread long orc_bcx_stat[4];

static uint32_t xs = 0x9E3779B9u;
static uint32_t xorshift(void) { xs ^= xs << 13; xs ^= xs >> 17; xs ^= xs << 5; return xs; }

int main(int argc, char **argv)
{
    const int W = 8192, H = 8192;
    const int rows = argc > 1 ? atoi(argv[1]) : 16;
    /* G1: gradient + xorshift noise in [-8, 8], row-major */
    uint8_t *img = malloc((size_t)W * H * 4);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            uint8_t *p = img + ((size_t)y * W + x) * 4;
            const int base[3] = {x * 255 / (W - 1), y * 255 / (H - 1), (x + y) * 255 / (W + H - 2)};
            const int nz = (int)(xorshift() % 17) - 8;
            for (int c = 0; c < 3; ++c) {
                int v = base[c] + nz;
                p[c] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
            }
            p[3] = 255;
        }
    long it3 = 0, it4 = 0, w3 = 0, w4 = 0, blocks = 0, waves = 0, skip4 = 0, lane4 = 0;
    long hist3[16] = {0}, hist4[16] = {0};
    for (int r = 0; r < rows; ++r) {
        const int by = (int)((long)r * (H / 4) / rows);
        for (int wx = 0; wx < W / 4; wx += 64) {
            long m3 = 0, m4 = 0, any4 = 0;
            for (int bx = wx; bx < wx + 64; ++bx) {
                float blk[64];
                orc_load_block_rgba8(img, W, H, 4, bx, by, 1, blk);
                orc_bcx_stat[0] = orc_bcx_stat[1] = 0;
                uint8_t out[8];
                orc_bc1_block(blk, 1, 128 / 255.0f, out);
                const long a = orc_bcx_stat[0], b = orc_bcx_stat[1];
                it3 += a;
                it4 += b;
                hist3[a < 15 ? a : 15]++;
                hist4[b < 15 ? b : 15]++;
                m3 = a > m3 ? a : m3;
                m4 = b > m4 ? b : m4;
                blocks++;
                if (b) { any4 = 1; lane4++; } else skip4++;
            }
            w3 += m3;
            w4 += m4;
            waves++;
            (void)any4;
        }
    }
    printf("blocks %ld waves %ld\n", blocks, waves);
    printf("3-colour axis loop: %.3f iterations per block, wave max %.3f -> lane utilisation %.1f %%\n",
           (double)it3 / blocks, (double)w3 / waves, 100.0 * it3 / (64.0 * w3));
    printf("4-colour axis loop: %.3f iterations per block, wave max %.3f -> lane utilisation %.1f %% "
           "(%ld blocks skip it: e3 == 0 or small)\n",
           (double)it4 / blocks, (double)w4 / waves, 100.0 * it4 / (64.0 * w4), skip4);
    printf("histogram 3-colour:");
    for (int i = 0; i < 16; ++i) printf(" %ld", hist3[i]);
    printf("\nhistogram 4-colour:");
    for (int i = 0; i < 16; ++i) printf(" %ld", hist4[i]);
    printf("\n");
    return 0;
}

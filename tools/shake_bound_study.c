/* ep_shaker_d corner-walk study for round 6 (oracle ORC_STATS counters 38-58):
 * round-two share of walked passes, and how many walked passes a per-channel
 * separable lower bound (every channel picks its own combo and cluster) would
 * skip, over block rows of the 8192^2 G1 texture.
 *   gcc -O2 -DORC_STATS -ffp-contract=off -I oracle tools/shake_bound_study.c oracle/orc_*.c -lm -lpthread -o /tmp/sbs
 *   /tmp/sbs <rows> <threads>      (profiles/r06_shake_bound_study.txt: 4 rows) */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include "bcn_oracle.h"
extern unsigned long long orc_stats[9][64];
static uint32_t xs = 0x9E3779B9u;
static uint32_t xorshift(void) { xs ^= xs << 13; xs ^= xs >> 17; xs ^= xs << 5; return xs; }
int main(int argc, char **argv)
{
    const int W = 8192, H = 8192;
    const int rows = argc > 1 ? atoi(argv[1]) : 2, threads = argc > 2 ? atoi(argv[2]) : 8;
    uint8_t *img = malloc((size_t)W * H * 4);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            uint8_t *p = img + ((size_t)y * W + x) * 4;
            const int base[3] = {x * 255 / (W - 1), y * 255 / (H - 1), (x + y) * 255 / (W + H - 2)};
            const int nz = (int)(xorshift() % 17) - 8;
            for (int c = 0; c < 3; ++c) { int v = base[c] + nz; p[c] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }
            p[3] = 255;
        }
    uint8_t *dst = malloc((size_t)(W / 4) * 16);
    for (int r = 0; r < rows; ++r) {
        const int by = (int)((long)r * (H / 4) / rows);
        orc_encode_image_bc7(img, W, H, 1, 4, by, 1, threads, 1.0f, 0xff, dst, NULL);
    }
    for (int m = 0; m < 9; ++m) {
        unsigned long long *S = orc_stats[m];
        if (!S[38]) continue;
        printf("mode %2d: calls %llu rounds2 %llu | walked %llu: min<thr %.1f%%, min>=thr %.1f%%, LBall>=thr %.1f%%, LB2>=thr %.1f%% | walked r1 %llu r2 %llu\n",
               m == 8 ? -1 : m, S[0], S[55], S[38], 100.0 * S[39] / S[38], 100.0 * S[53] / S[38], 100.0 * S[52] / S[38],
               100.0 * S[54] / S[38], S[57], S[58]);
    }
    for (int m = 0; m < 9; ++m) {
        unsigned long long *S = orc_stats[m];
        if (!S[38]) continue;
        printf("mode %2d: walked %llu texels %llu; texels used natural %.2f distdesc %.2f mincontrib %.2f per walked pass\n",
               m == 8 ? -1 : m, S[38], S[48], (double)S[49] / S[38], (double)S[50] / S[38], (double)S[51] / S[38]);
    }
    return 0;
}

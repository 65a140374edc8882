/* Walked (non-repeated) ep_shaker_d corner passes per expansion, per BC7 mode,
 * from the oracle's ORC_STATS counters (slots 17..21: 0, 1, 2, 3, >=4 walked
 * passes; 36/37: passes / repeated passes) over block rows of the 8192^2 G1
 * texture -- the input to pairing two passes of one expansion in one wave walk.
 *   gcc -O2 -DORC_STATS -ffp-contract=off -I oracle tools/bc7_pass_study.c oracle/orc_*.c -lm -lpthread -o /tmp/bc7p
 *   /tmp/bc7p <rows> <threads> */
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
            for (int c = 0; c < 3; ++c) {
                int v = base[c] + nz;
                p[c] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
            }
            p[3] = 255;
        }
    uint8_t *dst = malloc((size_t)(W / 4) * 16);
    for (int r = 0; r < rows; ++r) {
        const int by = (int)((long)r * (H / 4) / rows);
        orc_encode_image_bc7(img, W, H, 1, 4, by, 1, threads, 1.0f, 0xff, dst, NULL);
    }
    for (int m = 0; m < 9; ++m) {
        unsigned long long tot = 0;
        for (int k = 17; k <= 21; ++k) tot += orc_stats[m][k];
        if (!tot) continue;
        printf("mode %d: expansions %llu, passes %llu (repeated %llu); walked passes per expansion:", m == 8 ? -1 : m,
               tot, orc_stats[m][36], orc_stats[m][37]);
        for (int k = 17; k <= 21; ++k) printf(" %d:%.1f%%", k - 17, 100.0 * orc_stats[m][k] / tot);
        printf("\n");
    }
    return 0;
}

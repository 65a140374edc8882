/* Early-exit study for the BC1 kernel's 8x8 endpoint candidates (RampSrchW,
 * amd_bcx_body.cpp:398-435; gic_bcx.hip fit_endpoints, lane path).  A wave runs
 * 64 blocks (consecutive blocks of a block row) in lockstep: candidate c of
 * axis iteration `it` of the 3- or 4-colour search is one step for every lane
 * still in that loop.  Today the kernel evaluates entries 0..7, then 8..15
 * unless every active lane's running sum has reached its best error so far.
 * This counts, with the oracle's running sums (ORC_STATS hook), the entries a
 * wave evaluates under
 *   A  the current scheme,
 *   B  entries past the wave's largest unique-colour count skipped (they add +0),
 *   C  B + the cut bound strengthened by the remaining entries' perpendicular
 *      errors (each later term is >= its perr, so running + sum(perr rest)
 *      bounds the total from below), checkpoints after 4, 8 and 12 entries.
 *   gcc -O2 -DORC_STATS -ffp-contract=off -I oracle tools/bc1_cut_study.c oracle/orc_*.c -lm -lpthread -o /tmp/bc1c
 *   /tmp/bc1c <rows>   (rows of the 8192^2 G1 texture, every 2048/rows-th row) */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
#include "bcn_oracle.h"

extern void (*orc_bcx_ramp_hook)(const float run[16], const float perr[16], float maxerr, int ncol, int n);

typedef struct {
    float run[16], sfx[17];   /* sfx[k] = sum of perr[k..] (float, rounded down below) */
    float maxerr;
    int ncol, n;
} Call;

enum { kMaxCalls = 64 * 64 };
static Call calls[64][kMaxCalls];
static int ncalls[64];
static int cur;

static void hook(const float run[16], const float perr[16], float maxerr, int ncol, int n)
{
    Call *c = &calls[cur][ncalls[cur]++];
    memcpy(c->run, run, sizeof(c->run));
    double s = 0;
    c->sfx[16] = 0;
    for (int k = 15; k >= 0; --k) {
        s += k < ncol ? perr[k] : 0.f;
        c->sfx[k] = (float)(s * (1.0 - 1.0 / (1 << 20)));
    }
    c->maxerr = maxerr;
    c->ncol = ncol;
    c->n = n;
}

static uint32_t xs = 0x9E3779B9u;
static uint32_t xorshift(void) { xs ^= xs << 13; xs ^= xs >> 17; xs ^= xs << 5; return xs; }

int main(int argc, char **argv)
{
    const int W = 8192, H = 8192;
    const int rows = argc > 1 ? atoi(argv[1]) : 16;
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
    orc_bcx_ramp_hook = hook;
    double costA = 0, costB = 0, costC = 0, costC8 = 0, steps = 0, cutA = 0, cutC[3] = {0, 0, 0};
    for (int r = 0; r < rows; ++r) {
        const int by = (int)((long)r * (H / 4) / rows);
        for (int wx = 0; wx < W / 4; wx += 64) {
            int nmax = 0;
            for (int l = 0; l < 64; ++l) {
                float blk[64];
                orc_load_block_rgba8(img, W, H, 4, wx + l, by, 1, blk);
                cur = l;
                ncalls[l] = 0;
                uint8_t out[8];
                orc_bc1_block(blk, 1, 128 / 255.0f, out);
                for (int k = 0; k < ncalls[l]; ++k) nmax = calls[l][k].ncol > nmax ? calls[l][k].ncol : nmax;
            }
            /* align lanes by (n, call index within that n's calls) */
            for (int n = 3; n <= 4; ++n) {
                int pos[64], len[64], maxlen = 0;
                for (int l = 0; l < 64; ++l) {
                    pos[l] = -1;
                    len[l] = 0;
                    for (int k = 0; k < ncalls[l]; ++k)
                        if (calls[l][k].n == n) {
                            if (pos[l] < 0) pos[l] = k;
                            len[l]++;
                        }
                    maxlen = len[l] > maxlen ? len[l] : maxlen;
                }
                for (int t = 0; t < maxlen; ++t) {
                    int allA = 1, allC[3] = {1, 1, 1}, active = 0;
                    for (int l = 0; l < 64; ++l) {
                        if (t >= len[l]) continue;
                        active++;
                        const Call *c = &calls[l][pos[l] + t];
                        if (!(c->run[7] >= c->maxerr)) allA = 0;
                        for (int q = 0; q < 3; ++q) {
                            const int k = 4 * (q + 1);
                            if (!(c->run[k - 1] + c->sfx[k] >= c->maxerr)) allC[q] = 0;
                        }
                    }
                    if (!active) continue;
                    steps++;
                    costA += allA ? 8 : 16;
                    cutA += allA;
                    costB += allA ? 8 : nmax;
                    int e = nmax;
                    for (int q = 0; q < 3; ++q)
                        if (allC[q] && 4 * (q + 1) < e) {
                            e = 4 * (q + 1);
                            cutC[q]++;
                            break;
                        }
                    costC += e;
                    costC8 += allC[1] ? 8 : nmax;
                }
            }
        }
    }
    printf("wave candidate steps %.0f\n", steps);
    printf("A current        : %.3f entries per step (cut at 8: %.1f %%)\n", costA / steps, 100 * cutA / steps);
    printf("B + nmax skip    : %.3f\n", costB / steps);
    printf("C + perr bound   : %.3f (cut at 4/8/12: %.1f / %.1f / %.1f %%)\n", costC / steps,
           100 * cutC[0] / steps, 100 * cutC[1] / steps, 100 * cutC[2] / steps);
    printf("C8 (bound, one checkpoint at 8): %.3f\n", costC8 / steps);
    return 0;
}

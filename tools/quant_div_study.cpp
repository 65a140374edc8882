// Lane divergence of k_quant_sub (host study): runs the product's register-
// resident optQuantAnD_d (bc7_quant.inc) over the distinct subset problems of
// modes 0-3 of real blocks, counts the steps (requantisation passes + lattice
// roundings) of each, and compares the sum over 64-lane waves of the longest
// lane (what a wave costs) with the mean (what a perfectly balanced wave
// would cost), for the kernel's lane order (block-major, problem-minor) and
// for problem-major orders.
//   g++ -O2 -o /tmp/qd/study tools/quant_div_study.cpp && /tmp/qd/study texels.u32 nblocks
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <cmath>
static long g_steps = 0;
#define GIC_QUANT_STEP_HOOK (++g_steps)
#include "../gfx_imagecompress_amd/csrc/bc7_quant.inc"
#include "../gfx_imagecompress_amd/csrc/bc7_tables.h"

int main(int argc, char **argv)
{
    FILE *f = fopen(argv[1], "rb");
    const int nb = atoi(argv[2]);
    std::vector<uint32_t> px((size_t)nb * 16);
    if (fread(px.data(), 4, px.size(), f) != px.size()) return 1;
    std::vector<uint32_t> prob;
    for (int pass = 0; pass < 2; ++pass)
        for (int task = 0; task < 208; ++task) {
            const int mode = task < 16 ? 0 : task < 80 ? 1 : task < 144 ? 2 : 3;
            const int part = task < 16 ? task : task < 80 ? task - 16 : task < 144 ? task - 80 : task - 144;
            const int clog = (mode <= 1) ? 3 : 2;
            if ((clog == 3) != (pass == 0)) continue;
            const int subsets = (mode == 0 || mode == 2) ? 3 : 2;
            const uint32_t shape = subsets == 3 ? kBc7Shape3[part] : kBc7Shape2[part];
            for (int j = 0; j < subsets; ++j) {
                uint32_t m = 0;
                for (int t = 0; t < 16; ++t) m |= (((shape >> (2 * t)) & 3u) == (uint32_t)j ? 1u : 0u) << t;
                const uint32_t key = m | (uint32_t)clog << 16;
                if (std::find(prob.begin(), prob.end(), key) == prob.end()) prob.push_back(key);
            }
        }
    const int nu = (int)prob.size();
    std::vector<long> steps((size_t)nb * nu);
    for (int b = 0; b < nb; ++b)
        for (int u = 0; u < nu; ++u) {
            int idx[16];
            g_steps = 0;
            opt_quant_mask<3>(&px[(size_t)b * 16], prob[u] & 0xFFFF, 1 << (prob[u] >> 16), idx);
            steps[(size_t)b * nu + u] = g_steps;
        }
    auto waves = [&](auto order) {
        long sum = 0, wmax = 0;
        const size_t N = steps.size();
        for (size_t w = 0; w < N; w += 64) {
            long m = 0;
            for (size_t l = w; l < std::min(N, w + 64); ++l) {
                const long s = steps[order(l)];
                sum += s;
                m = std::max(m, s);
            }
            wmax += m * (long)std::min<size_t>(64, N - w);
        }
        return std::pair<long, long>(sum, wmax);
    };
    auto r0 = waves([&](size_t l) { return l; });
    auto r1 = waves([&](size_t l) { const size_t u = l / nb, b = l % nb; return b * nu + u; });
    std::vector<size_t> srt(steps.size());
    for (size_t i = 0; i < srt.size(); ++i) srt[i] = i;
    std::sort(srt.begin(), srt.end(), [&](size_t a, size_t c) { return steps[a] < steps[c]; });
    auto r2 = waves([&](size_t l) { return srt[l]; });
    long mx = *std::max_element(steps.begin(), steps.end());
    printf("nu %d problems %zu mean steps %.2f max %ld\n", nu, steps.size(), (double)r0.first / steps.size(), mx);
    printf("block-major (kernel): lane efficiency %.3f\n", (double)r0.first / r0.second);
    printf("problem-major:        lane efficiency %.3f\n", (double)r1.first / r1.second);
    printf("sorted by steps:      lane efficiency %.3f\n", (double)r2.first / r2.second);
    std::vector<long> hist(12, 0);
    for (long s : steps) { int k = 0; while ((1L << k) < s && k < 11) ++k; hist[k]++; }
    for (int k = 0; k < 12; ++k) printf("  steps <= %5ld: %ld\n", 1L << k, hist[k]);
    return 0;
}

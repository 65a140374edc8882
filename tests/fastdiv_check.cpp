// Host check of gic::div3_rn (csrc/gic_fastdiv.h) against IEEE float division:
// every STRIDE-th float bit pattern (argv[1]), infinities and NaNs skipped (the
// BC1 search never divides them).  The GPU check over all 2^32 inputs, including
// rcp_rn, is tools/rcp_check.hip.
#define GIC_FASTDIV_HOST
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../gfx_imagecompress_amd/csrc/gic_fastdiv.h"

int main(int argc, char **argv)
{
    const uint64_t stride = argc > 1 ? strtoull(argv[1], nullptr, 10) : 7;
    uint64_t n = 0, bad = 0;
    for (uint64_t u = 0; u < (1ull << 32); u += stride) {
        const uint32_t b = (uint32_t)u;
        float d;
        memcpy(&d, &b, 4);
        if (!std::isfinite(d)) continue;
        ++n;
        const float q = gic::div3_rn(d), r = d / 3.0f;
        if (memcmp(&q, &r, 4) != 0) ++bad;
    }
    printf("%llu/%llu mismatches\n", (unsigned long long)bad, (unsigned long long)n);
    return bad ? 1 : 0;
}

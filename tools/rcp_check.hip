// Exhaustive check, on the GPU, of the two fast float divisions the BC1 kernel
// uses in place of the IEEE division sequence (csrc/gic_bcx.hip div3_rn /
// rcp_rn): for every float bit pattern, RN(d / 3) by one multiply and two FMAs
// and RN(1 / s) by v_rcp_f32 plus one FMA Newton step, against the compiler's
// correctly rounded division (built with the library's numerics flags).
//   hipcc --offload-arch=gfx950 <NUMERICS> tools/rcp_check.hip -o tools/rcp_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include "../gfx_imagecompress_amd/csrc/gic_fastdiv.h"

__global__ void check(unsigned long long *bad, unsigned *first)
{
    const unsigned long long n = 1ull << 32;
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        const float x = __uint_as_float((unsigned)i);
        const float a = gic::div3_rn(x), b = x / 3.0f;   // NaN inputs: both NaN
        if (__float_as_uint(a) != __float_as_uint(b) && !(a != a && b != b)) {
            atomicAdd(&bad[0], 1ull);
            atomicMin(&first[0], (unsigned)i);
        }
        const float c = gic::rcp_rn(x), d = 1.0f / x;
        if (__float_as_uint(c) != __float_as_uint(d) && !(c != c && d != d)) {
            atomicAdd(&bad[1], 1ull);
            atomicMin(&first[1], (unsigned)i);
        }
    }
}

int main()
{
    unsigned long long *bad;
    unsigned *first;
    if (hipMalloc(&bad, 16) != hipSuccess || hipMalloc(&first, 8) != hipSuccess) return 2;
    hipMemset(bad, 0, 16);
    hipMemset(first, 0xff, 8);
    check<<<8192, 256>>>(bad, first);
    unsigned long long hb[2];
    unsigned hf[2];
    if (hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    hipMemcpy(hf, first, 8, hipMemcpyDeviceToHost);
    printf("div3_rn: %llu mismatches (first 0x%08x); rcp_rn: %llu mismatches (first 0x%08x) over all 2^32 inputs\n",
           hb[0], hf[0], hb[1], hf[1]);
    return (hb[0] || hb[1]) ? 1 : 0;
}

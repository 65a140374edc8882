// Check of the product's register-resident quantiser
// (gfx_imagecompress_amd/csrc/bc7_quant.inc) against the oracle's
// optQuantAnD_d restatement, on random subsets of random integer blocks, on
// gradient blocks (which drive the 200-iteration path) and on replicated-channel
// blocks (the dual-index alpha half).  Built with g++ it runs the quantiser on
// the host; built with hipcc (-x hip) it runs it on the GPU, once with a runtime
// texel mask and once with the compile-time full mask the dual-index kernel
// uses.  Driven by tests/test_quant_equiv.py.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GIC_QUANT_FF_HOOK
#else
static long g_ff = 0;
#define GIC_QUANT_FF_HOOK (++g_ff)
#endif
#include "../gfx_imagecompress_amd/csrc/bc7_quant.inc"
extern "C" double orc_bc7_opt_quant(const double *data4, int n, int ncl, int *index, int dim);

struct Trial {
    uint32_t px[16];
    uint32_t mask;
    int dim, ncl;
};

static uint32_t rng = 12345;
static uint32_t nextr() { rng ^= rng << 13; rng ^= rng >> 17; rng ^= rng << 5; return rng; }

// Every third trial runs the compacted form (SelPrefix, k_quant_sub): the
// subset's texels moved to slots 0..n-1, indices scattered back.
template <int DIM>
GIC_HD double quant_prefix(const uint32_t px[16], uint32_t mask, int ncl, int idx[16])
{
    uint32_t pc[16];
    int ic[16], n = 0;
    for (int i = 0; i < 16; ++i) pc[i] = 0;
    for (int i = 0; i < 16; ++i)
        if ((mask >> i) & 1u) pc[n++] = px[i];
    const double e = opt_quant_sel<DIM>(pc, SelPrefix{n}, ncl, ic);
    for (int i = 0, k = 0; i < 16; ++i) idx[i] = ((mask >> i) & 1u) ? ic[k++] : 0;
    return e;
}

#if defined(__HIPCC__)
__global__ void k_equiv(const Trial *tr, int n, double *err, int *idx)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    uint32_t px[16];
    for (int i = 0; i < 16; ++i) px[i] = tr[t].px[i];
    int id[16];
    double e;
    if (t % 3 == 2)
        e = tr[t].dim == 3 ? quant_prefix<3>(px, tr[t].mask, tr[t].ncl, id) : quant_prefix<4>(px, tr[t].mask, tr[t].ncl, id);
    else if (tr[t].mask == 0xffffu && tr[t].dim == 3)
        e = opt_quant_mask<3>(px, 0xffffu, tr[t].ncl, id);   // constant mask, as k_dual_quant
    else if (tr[t].dim == 3)
        e = opt_quant_mask<3>(px, tr[t].mask, tr[t].ncl, id);
    else
        e = opt_quant_mask<4>(px, tr[t].mask, tr[t].ncl, id);
    err[t] = e;
    for (int i = 0; i < 16; ++i) idx[t * 16 + i] = id[i];
}
#endif

int main(int argc, char **argv)
{
    const int trials = argc > 1 ? atoi(argv[1]) : 20000;
    std::vector<Trial> tr(trials);
    for (int t = 0; t < trials; ++t) {
        const int kind = t % 4;
        for (int i = 0; i < 16; ++i) {
            uint32_t v = 0;
            for (int c = 0; c < 4; ++c) {
                int x;
                if (kind == 0) x = nextr() & 255;
                else if (kind == 1) x = ((i & 3) * 3 + (i >> 2) * (c + 1) + (int)(nextr() % 3)) & 255;   // gentle gradient
                else if (kind == 2) x = 100 + (int)((i & 3) * (c + 2)) + (int)(i >> 2);
                else x = (c == 0) ? (int)(nextr() & 255) : (int)(v & 255);   // replicated channel (dual-index alpha)
                v |= (uint32_t)x << (8 * c);
            }
            tr[t].px[i] = v;
        }
        uint32_t mask = (nextr() & 0xffff) | (1u << (nextr() & 15));
        if (t % 5 == 0) mask = 0xffff;
        tr[t].mask = mask;
        tr[t].dim = ((t >> 2) & 1) ? 4 : 3;
        tr[t].ncl = 1 << (2 + (int)(nextr() % 3));
    }
    std::vector<double> err(trials);
    std::vector<int> idx((size_t)trials * 16);
#if defined(__HIPCC__)
    Trial *dtr;
    double *derr;
    int *didx;
    if (hipMalloc(&dtr, sizeof(Trial) * trials) != hipSuccess || hipMalloc(&derr, 8 * trials) != hipSuccess ||
        hipMalloc(&didx, 64 * trials) != hipSuccess) {
        printf("hipMalloc failed\n");
        return 2;
    }
    hipMemcpy(dtr, tr.data(), sizeof(Trial) * trials, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_equiv, dim3((trials + 127) / 128), dim3(128), 0, 0, dtr, trials, derr, didx);
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel failed\n");
        return 2;
    }
    hipMemcpy(err.data(), derr, 8 * trials, hipMemcpyDeviceToHost);
    hipMemcpy(idx.data(), didx, 64 * trials, hipMemcpyDeviceToHost);
    const long ff = -1;
#else
    for (int t = 0; t < trials; ++t)
        if (t % 3 == 2)
            err[t] = tr[t].dim == 3 ? quant_prefix<3>(tr[t].px, tr[t].mask, tr[t].ncl, &idx[t * 16])
                                    : quant_prefix<4>(tr[t].px, tr[t].mask, tr[t].ncl, &idx[t * 16]);
        else
            err[t] = tr[t].dim == 3 ? opt_quant_mask<3>(tr[t].px, tr[t].mask, tr[t].ncl, &idx[t * 16])
                                    : opt_quant_mask<4>(tr[t].px, tr[t].mask, tr[t].ncl, &idx[t * 16]);
    const long ff = g_ff;
#endif
    int bad = 0;
    for (int t = 0; t < trials; ++t) {
        double data[64];
        int n = 0, ridx[16];
        for (int i = 0; i < 16; ++i)
            if ((tr[t].mask >> i) & 1u) {
                for (int c = 0; c < 4; ++c) data[n * 4 + c] = (double)((tr[t].px[i] >> (8 * c)) & 255u);
                n++;
            }
        const double re = orc_bc7_opt_quant(data, n, tr[t].ncl, ridx, tr[t].dim);
        bool ok = err[t] == re;
        for (int i = 0, k = 0; i < 16; ++i)
            if ((tr[t].mask >> i) & 1u) ok = ok && idx[t * 16 + i] == ridx[k++];
        if (!ok) {
            if (bad < 10) {
                printf("mismatch trial %d kind %d dim %d ncl %d n %d: %.17g vs %.17g\n  got", t, t % 4, tr[t].dim,
                       tr[t].ncl, n, err[t], re);
                for (int i = 0; i < 16; ++i)
                    if ((tr[t].mask >> i) & 1u) printf(" %d", idx[t * 16 + i]);
                printf("\n  ref");
                for (int k = 0; k < n; ++k) printf(" %d", ridx[k]);
                printf("\n");
            }
            bad++;
        }
    }
    printf("%d/%d mismatches (%ld fast-forwarded runs)\n", bad, trials, ff);
    return bad != 0;
}

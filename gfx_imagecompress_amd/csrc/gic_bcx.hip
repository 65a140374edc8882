// gic_bcx.hip -- BC1 and BC4/BC5 block search for gfx950 (MI355X).
//
// Algorithm: the AMD Compressonator DXT search used by the reference
// (src/amd_bcx_body.cpp, src/amd_bcx_helpers.cpp): PCA axis, 8x8 endpoint
// ramp search on the projected axis with axis re-fitting, 565 grid snap,
// per-channel 3x3 refinement, weighted clustering; BC4 is the 1-D window
// search + hill climb of CompBlock1.  Results are bit-exact with the
// reference: every float expression keeps the reference's types and
// association order and the file is compiled with -ffp-contract=off.
//
// Mapping: one lane per 4x4 block (the work per block is a serial chain of
// small data-dependent loops); 256-lane workgroups; the grid covers every
// block of the launch.  Source texels are read as 16-byte rows so a wave's
// 64 adjacent blocks issue fully coalesced 1 KiB row loads; each lane writes
// one 8-byte (BC1/BC4) or 16-byte (BC5) block, coalesced across the wave.
// The early-out of RampSrchW / RmpSrch1 is replaced by full evaluation: the
// per-colour error terms are non-negative, so the partial sums are monotone
// and "first strictly smaller" selection is unchanged.

#include "gic_common.h"
#include "gic_fastdiv.h"

namespace gic {
namespace bcx {

enum { CH_B = 0, CH_G = 1, CH_R = 2, CH_A = 3 };

__device__ __forceinline__ int chan_bits(int ch) { return ch == CH_G ? 6 : 5; }

// MkRmpOnGrid, amd_bcx_body.cpp:122-151
__device__ void snap_grid(float out[3][2], const float in[3][2])
{
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        const float f1 = (float)(1 << chan_bits(ch));
        const float f0 = (float)(1 << (8 - chan_bits(ch)));
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            float v = floorf(in[ch][e]);
            if (v <= 0.f) {
                v = 0.f;
            } else {
                v += floorf(128.f / f1) - floorf(v / f1);
                v = minr(v, 255.f);
            }
            out[ch][e] = floorf(v / f0) * f0;
        }
    }
}

// MkWkRmpPts, amd_bcx_body.cpp:157-181
__device__ __forceinline__ bool expand_grid(float out[3][2], const float in[3][2])
{
    bool flat = true;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) flat &= (in[ch][0] == in[ch][1]);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        const float f = (float)(1 << chan_bits(ch));
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            float v = in[ch][e] + floorf(in[ch][e] / f);
            v = maxr(v, 0.f);
            out[ch][e] = minr(v, 255.f);
        }
    }
    return flat;
}

// BldClrRmp, amd_bcx_body.cpp:188-197 (n is 3 or 4)
// (x / (N - 1) is the IEEE quotient either way: N = 3 halves exactly, N = 4 takes
// div3_rn, gic_fastdiv.h)
template <int N>
__device__ __forceinline__ float div_nm1(float x)
{
    return N == 4 ? div3_rn(x) : x / (float)(N - 1);
}

template <int N>
__device__ __forceinline__ void chan_ramp(float r[4], const float ends[2])
{
    const float rnd = (N == 4) ? 1.f : 0.f;
    r[0] = ends[0];
    r[N - 1] = ends[1];
    if (N & 1) r[N] = 1000000.f;
#pragma unroll
    for (int e = 1; e < N - 1; ++e)
        r[e] = floorf(div_nm1<N>(r[0] * (float)(N - 1 - e) + r[N - 1] * (float)e + rnd));
}

// Unique colours of a block (B,G,R x255 as floats, sorted as QSortFloatCmp)
// with repeat counts.  Slots i >= n read as colour 0 with count 0, so sums
// weighted by the count are unchanged by them.  Every loop over colours is a
// fixed 16-step unrolled loop, which keeps the per-block arrays in VGPRs.
//   ColB: 8-bit sources -- one word per colour, bytes B, G, R, count.
//   ColF: float sources (block API).
//   blk(i, ch) = c(i, ch) / 255.f (FindAxis' input scale); ColB reads it from
//   the workgroup's byte -> v / 255.0f table (the same value).
// Byte -> float conversions as opaque single instructions: the compiler would
// otherwise hoist all 48 of them out of the search loops and run out of VGPRs.
__device__ __forceinline__ float ubyte_f(uint32_t w, int b)
{
    float r;
    switch (b) {
    case 0: asm volatile("v_cvt_f32_ubyte0 %0, %1" : "=v"(r) : "v"(w)); break;
    case 1: asm volatile("v_cvt_f32_ubyte1 %0, %1" : "=v"(r) : "v"(w)); break;
    case 2: asm volatile("v_cvt_f32_ubyte2 %0, %1" : "=v"(r) : "v"(w)); break;
    default: asm volatile("v_cvt_f32_ubyte3 %0, %1" : "=v"(r) : "v"(w)); break;
    }
    return r;
}

// LDS through its own address space (ds_read / ds_write).  The tables used to
// be reached through volatile generic pointers to keep the compiler from
// hoisting their loads into registers; volatile generic accesses compile to
// flat loads with the cache-bypass bits, each followed by a vmcnt(0) wait (the
// address-space inference leaves volatile accesses alone).  Now the address
// goes through an empty asm at every use: as opaque to the optimiser, but an
// ordinary LDS load the scheduler can batch.
typedef __attribute__((address_space(3))) float lds_f32_t;
typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
__device__ __forceinline__ uint32_t lds_off(const void *p) { return (uint32_t)(uintptr_t)(const lds_f32_t *)p; }
__device__ __forceinline__ float lds_ld_f(uint32_t a)
{
    asm volatile("" : "+v"(a));
    return *(const lds_f32_t *)(size_t)a;
}
// base made opaque, the constant offset added after it (the ds_read offset
// field): an opaque base + offset address would be computed for every word up
// front and kept live -- the 3-wave BC1 build spilled those addresses
__device__ __forceinline__ uint32_t lds_ld_u(uint32_t base, uint32_t off)
{
    asm volatile("" : "+v"(base));
    return *(const lds_u32_t *)(size_t)(base + off);
}
__device__ __forceinline__ void lds_st_u(uint32_t a, uint32_t v) { *(lds_u32_t *)(size_t)a = v; }

struct ColB {
    static constexpr bool kRefine3 = false;
    uint32_t u[16];
    int n;
    uint32_t lut;   // LDS byte address of the 256-entry byte -> v / 255.0f table
    __device__ __forceinline__ float c(int i, int ch) const { return ubyte_f(u[i], ch); }
    __device__ __forceinline__ float rpt(int i) const { return ubyte_f(u[i], 3); }
    __device__ __forceinline__ float blk(int i, int ch) const { return lds_ld_f(lut + 4u * ((u[i] >> (8 * ch)) & 255u)); }
};
struct ColF {
    static constexpr bool kRefine3 = false;
    float cc[16][3], r[16];
    int n;
    __device__ __forceinline__ float c(int i, int ch) const { return cc[i][ch]; }
    __device__ __forceinline__ float rpt(int i) const { return r[i]; }
    __device__ __forceinline__ float blk(int i, int ch) const { return cc[i][ch] / 255.f; }
};
// ColB's words parked in LDS through the endpoint search (colour i of a lane at
// w[i * kLdsStride], lane-contiguous rows, so a wave's reads are conflict-free):
// the search loop needs only the projections, and 16 colour words held in
// VGPRs across it pushed the kernel past 3 waves/SIMD into scratch.  Volatile:
// every use re-reads, nothing is hoisted into registers.  Refine takes a
// register copy (regs()).
constexpr int kLdsStride = 256;
// S1: the kernel runs only RefinementSteps == 1 (the default), and Refine
// takes refine_pass3 alone -- with the general pass compiled in beside it the
// 3-wave kernel spilled (see refine_pass3)
template <bool S1>
struct ColLT {
    static constexpr bool kRefine3 = S1;
    uint32_t w;   // LDS byte address of this lane's colour 0
    int n;
    uint32_t lut;
    __device__ __forceinline__ uint32_t word(int i) const { return lds_ld_u(w, 4u * (uint32_t)(i * kLdsStride)); }
    __device__ __forceinline__ float c(int i, int ch) const { return ubyte_f(word(i), ch); }
    __device__ __forceinline__ float rpt(int i) const { return ubyte_f(word(i), 3); }
    __device__ __forceinline__ float blk(int i, int ch) const
    {
        return lds_ld_f(lut + 4u * ((word(i) >> (8 * ch)) & 255u));
    }
    __device__ __forceinline__ ColB regs() const
    {
        ColB r;
        r.lut = lut;
        r.n = n;
#pragma unroll
        for (int i = 0; i < 16; ++i) r.u[i] = word(i);
        return r;
    }
};
// ColF with FindAxis' inputs cc / 255.f divided once (the one-wave block kernels:
// the divisions recomputed in every axis iteration's projection and direction
// loops were a quarter of a BC1 block's search)
struct ColFW : ColF {
    float bk[16][3];
    float *urow;   // the wave's LDS rows: 16 x 8 colour words, then 32 + 64 floats of exchange
    __device__ __forceinline__ float blk(int i, int ch) const { return bk[i][ch]; }
};
template <class C> struct LaneRows { static constexpr bool v = false; };
template <> struct LaneRows<ColFW> { static constexpr bool v = true; };

__device__ __forceinline__ void wave_sync_lds()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ const ColB &regs(const ColB &u) { return u; }
__device__ __forceinline__ const ColF &regs(const ColF &u) { return u; }
__device__ __forceinline__ const ColFW &regs(const ColFW &u) { return u; }
template <bool S1>
__device__ __forceinline__ ColB regs(const ColLT<S1> &u) { return u.regs(); }

// ClstrErr (weighted), amd_bcx_body.cpp:214-255
template <int N, class Col>
__device__ __forceinline__ float ramp_fit_error(const Col &u, const float r[3][4], bool flat)
{
    const float w0 = 0.3086f, w1 = 0.6094f, w2 = 0.0820f;
    float err = 0.f;
    const int nr = flat ? 1 : N;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        float best = 99999999999.f;
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const float cr = u.c(i, CH_R), cg = u.c(i, CH_G), cb = u.c(i, CH_B);
            float d = (cr - r[CH_R][k]) * (cr - r[CH_R][k]) * w0 + (cg - r[CH_G][k]) * (cg - r[CH_G][k]) * w1 +
                      (cb - r[CH_B][k]) * (cb - r[CH_B][k]) * w2;
            best = (k < nr && d < best) ? d : best;
        }
        err += best * u.rpt(i);   // count 0 past n: adds +0
    }
    return err;
}

// ---- wave-cooperative searches (one 64-lane wave per block: small batches,
// the block-level entry points).  Every lane holds the block; a search's
// candidates are spread over the lanes and the sequential choice -- the first
// strictly smaller error in loop order -- is recovered by an (error, order)
// minimum over the wave.  Each candidate's error is the same function of the
// same floats as in the lane-per-block loop, so the blocks are bit-identical.

// (e, order) of the lane with the smallest e, ties to the smallest order; a lane
// without a candidate brings e = +inf
// Unsigned minimum over the wave: DPP inside each 16-lane row (quad_perm xor 1,
// xor 2, row_ror 4, 8), then the four rows' results by readlane.  The whole
// wave must be active (every call site is wave-uniform).
template <int CTRL>
__device__ __forceinline__ unsigned dpp_u(unsigned v)
{
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ unsigned wave_minu(unsigned v)
{
    v = min(v, dpp_u<0xB1>(v));
    v = min(v, dpp_u<0x4E>(v));
    v = min(v, dpp_u<0x124>(v));
    v = min(v, dpp_u<0x128>(v));
    const unsigned a = (unsigned)__builtin_amdgcn_readlane((int)v, 0), b = (unsigned)__builtin_amdgcn_readlane((int)v, 16),
                   c = (unsigned)__builtin_amdgcn_readlane((int)v, 32), d = (unsigned)__builtin_amdgcn_readlane((int)v, 48);
    return min(min(a, b), min(c, d));
}

// (e, o) lexicographic minimum over the wave, on every lane.  Every caller feeds
// a non-negative, non-NaN e (+inf for "no candidate": the NaN-rejecting tests sit
// before the call) and o >= 0, so float order is the bit patterns' unsigned
// order and the minimum does not depend on the reduction order: two DPP
// minima instead of six rounds of two ds_bpermute shuffles.  e + 0.0f maps -0
// to +0 (round to nearest; the build has no fast-math) so a -0 ties with +0 and
// the lower o wins, as a float compare would have it.
__device__ __forceinline__ void wave_argmin(float &e, int &o)
{
    const unsigned eb = __float_as_uint(e + 0.0f);
    const unsigned emin = wave_minu(eb);
    const unsigned om = wave_minu(eb == emin ? (unsigned)o : 0xffffffffu);
    e = __uint_as_float(emin);
    o = (int)om;
}

// Refine, amd_bcx_body.cpp:582-806 (R, then G, then B 3x3 jitter of both
// endpoints on the 565 grid; RefinementSteps = `steps`).  One pass per
// channel, a template on the channel so every index is static (a runtime
// channel loop does not unroll and turns each array access into selects).
template <int N, int CH, bool WAVE = false, class Col>
__device__ __forceinline__ void refine_pass(float cur[3][2], const float base[3][2], const Col &u, int lo, int hi,
                                            float &best)
{
    const float wr = 0.3086f, wg = 0.6094f, wb = 0.0820f;
    float wk[3][2], r[3][4], side[4][16];
    {
        const bool flat = expand_grid(wk, cur);
        (void)flat;
#pragma unroll
        for (int c = 0; c < 3; ++c) chan_ramp<N>(r[c], wk[c]);
    }
    if constexpr (WAVE && LaneRows<Col>::v) {
        // one-wave kernels: lane i < n forms colour i's side terms (the same
        // expressions), the wave reads the table back (entries past n: unused
        // by the count-0 colours, read as written or stale, multiplied by 0)
        const int L = (int)(threadIdx.x & 63u);
        float *y = u.urow + 160;
        if (L < u.n) {
            const float c0 = u.urow[L * 8 + 0], c1 = u.urow[L * 8 + 1], c2 = u.urow[L * 8 + 2];
            const float cc[3] = {c0, c1, c2};
#pragma unroll
            for (int k = 0; k < N; ++k) {
                float v;
                if (CH == CH_R) {
                    float dg = r[CH_G][k] - cc[CH_G], db = r[CH_B][k] - cc[CH_B];
                    v = dg * dg * wg + db * db * wb;
                } else if (CH == CH_G) {
                    float dr = r[CH_R][k] - cc[CH_R], db = r[CH_B][k] - cc[CH_B];
                    v = dr * dr * wr + db * db * wb;
                } else {
                    float dr = r[CH_R][k] - cc[CH_R], dg = r[CH_G][k] - cc[CH_G];
                    v = dr * dr * wr + dg * dg * wg;
                }
                y[L * 4 + k] = v;
            }
        }
        wave_sync_lds();
#pragma unroll
        for (int i = 0; i < 16; ++i)
#pragma unroll
            for (int k = 0; k < N; ++k) side[k][i] = i < u.n ? y[i * 4 + k] : 0.f;
    } else {
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int k = 0; k < N; ++k) {
            if (CH == CH_R) {
                float dg = r[CH_G][k] - u.c(i, CH_G), db = r[CH_B][k] - u.c(i, CH_B);
                side[k][i] = dg * dg * wg + db * db * wb;
            } else if (CH == CH_G) {
                float dr = r[CH_R][k] - u.c(i, CH_R), db = r[CH_B][k] - u.c(i, CH_B);
                side[k][i] = dr * dr * wr + db * db * wb;
            } else {
                float dr = r[CH_R][k] - u.c(i, CH_R), dg = r[CH_G][k] - u.c(i, CH_G);
                side[k][i] = dr * dr * wr + dg * dg * wg;
            }
        }
    }
    const float grid = (float)(1 << (8 - chan_bits(CH)));
    const float wc = (CH == CH_R) ? wr : (CH == CH_G) ? wg : wb;
    float b0 = base[CH][0], b1 = base[CH][1];
    if constexpr (WAVE) {
        // candidate t = (a - lo) * span + (b - lo) on lane t % 64
        const int span = hi - lo + 1, ln = (int)(threadIdx.x & 63u);
        float be = __builtin_huge_valf();
        int bo = 0x7fffffff;
        if constexpr (LaneRows<Col>::v) {
            if (span == 3) {
                // steps == 1: the 9 candidates x 16 colours on the lanes, each
                // (candidate, colour) term into an LDS row, then candidate t's
                // lane sums its 16 terms in colour order (the same additions)
                float *tm = u.urow + 224;
                const float *y = u.urow + 160;
                for (int q = ln; q < 144; q += 64) {
                    const int t = q >> 4, i = q & 15;
                    float c2[3][2], w2[3][2], rr[4];
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        c2[c][0] = cur[c][0];
                        c2[c][1] = cur[c][1];
                    }
                    c2[CH][0] = minr(maxr(base[CH][0] + (float)(lo + t / 3) * grid, 0.f), 255.f);
                    c2[CH][1] = minr(maxr(base[CH][1] + (float)(lo + t % 3) * grid, 0.f), 255.f);
                    const bool flat = expand_grid(w2, c2);
                    chan_ramp<N>(rr, w2[CH]);
                    const int nr = flat ? 1 : N;
                    float term = 0.f;
                    if (i < u.n) {
                        const float ci = u.urow[i * 8 + CH];
                        float m = 10000000.f;
#pragma unroll
                        for (int k = 0; k < N; ++k) {
                            float d = rr[k] - ci;
                            float e = y[i * 4 + k] + d * d * wc;
                            m = (k < nr) ? minr(m, e) : m;
                        }
                        term = m * u.urow[i * 8 + 3];
                    }
                    tm[q] = term;
                }
                wave_sync_lds();
                if (ln < 9) {
                    float mse = 0.f;
#pragma unroll
                    for (int i = 0; i < 16; ++i) mse += tm[ln * 16 + i];
                    if (mse < best) {
                        be = mse;
                        bo = ln;
                    }
                }
                wave_argmin(be, bo);
                if (bo != 0x7fffffff) {
                    b0 = minr(maxr(base[CH][0] + (float)(lo + bo / span) * grid, 0.f), 255.f);
                    b1 = minr(maxr(base[CH][1] + (float)(lo + bo % span) * grid, 0.f), 255.f);
                    best = be;
                }
                cur[CH][0] = b0;
                cur[CH][1] = b1;
                return;
            }
        }
        for (int t = ln; t < span * span; t += 64) {
            const int a = lo + t / span, b = lo + t % span;
            cur[CH][0] = minr(maxr(base[CH][0] + (float)a * grid, 0.f), 255.f);
            cur[CH][1] = minr(maxr(base[CH][1] + (float)b * grid, 0.f), 255.f);
            const bool flat = expand_grid(wk, cur);
            chan_ramp<N>(r[CH], wk[CH]);
            float mse = 0.f;
            const int nr = flat ? 1 : N;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                float m = 10000000.f;
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    float d = r[CH][k] - u.c(i, CH);
                    float e = side[k][i] + d * d * wc;
                    m = (k < nr) ? minr(m, e) : m;
                }
                mse += m * u.rpt(i);
            }
            if (mse < best && mse < be) {
                be = mse;
                bo = t;
            }
        }
        wave_argmin(be, bo);
        if (bo != 0x7fffffff) {
            b0 = minr(maxr(base[CH][0] + (float)(lo + bo / span) * grid, 0.f), 255.f);
            b1 = minr(maxr(base[CH][1] + (float)(lo + bo % span) * grid, 0.f), 255.f);
            best = be;
        }
        cur[CH][0] = b0;
        cur[CH][1] = b1;
        return;
    }
    for (int a = lo; a <= hi; ++a)
        for (int b = lo; b <= hi; ++b) {
            cur[CH][0] = minr(maxr(base[CH][0] + (float)a * grid, 0.f), 255.f);
            cur[CH][1] = minr(maxr(base[CH][1] + (float)b * grid, 0.f), 255.f);
            const bool flat = expand_grid(wk, cur);
            chan_ramp<N>(r[CH], wk[CH]);
            float mse = 0.f;
            const int nr = flat ? 1 : N;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                float m = 10000000.f;
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    float d = r[CH][k] - u.c(i, CH);
                    float e = side[k][i] + d * d * wc;
                    m = (k < nr) ? minr(m, e) : m;
                }
                mse += m * u.rpt(i);   // count 0 past n: adds +0
            }
            if (mse < best) {
                b0 = cur[CH][0];
                b1 = cur[CH][1];
                best = mse;
            }
        }
    cur[CH][0] = b0;
    cur[CH][1] = b1;
}

// The same pass for steps == 1 (the default: a, b in {-1, 0, 1}) over the
// LDS-parked colours (ColL), loops swapped: the nine candidates' ramps are
// built first, then one sweep over the block's colours -- a rolled loop, one
// LDS word per colour, n iterations -- accumulates all nine errors (each still
// summed in colour order; colours past n add +0), and the first strictly
// smaller candidate in (a, b) order wins as before.  Only one colour's N side
// terms are live instead of all 16 x N, which pushed the 3-wave BC1 kernel
// into scratch spills (32 B written per block).
template <int N, int CH>
__device__ __forceinline__ void refine_pass3(float cur[3][2], const float base[3][2], const ColLT<true> &u,
                                             float &best)
{
    const float wr = 0.3086f, wg = 0.6094f, wb = 0.0820f;
    float wk[3][2], r[3][4];
    {
        const bool flat = expand_grid(wk, cur);
        (void)flat;
#pragma unroll
        for (int c = 0; c < 3; ++c) chan_ramp<N>(r[c], wk[c]);
    }
    const float grid = (float)(1 << (8 - chan_bits(CH)));
    const float wc = (CH == CH_R) ? wr : (CH == CH_G) ? wg : wb;
    float rc[9][4], e0[9], e1[9], mse[9];
    bool flt[9];
#pragma unroll
    for (int ab = 0; ab < 9; ++ab) {
        const int a = ab / 3 - 1, b = ab % 3 - 1;
        cur[CH][0] = minr(maxr(base[CH][0] + (float)a * grid, 0.f), 255.f);
        cur[CH][1] = minr(maxr(base[CH][1] + (float)b * grid, 0.f), 255.f);
        e0[ab] = cur[CH][0];
        e1[ab] = cur[CH][1];
        flt[ab] = expand_grid(wk, cur);
        chan_ramp<N>(rc[ab], wk[CH]);
        mse[ab] = 0.f;
    }
#pragma unroll 1
    for (int i = 0; i < u.n; ++i) {
        const uint32_t wd = u.word(i);
        const float cr = ubyte_f(wd, CH_R), cg = ubyte_f(wd, CH_G), cb = ubyte_f(wd, CH_B), rp = ubyte_f(wd, 3);
        float side[4];
#pragma unroll
        for (int k = 0; k < N; ++k) {
            if (CH == CH_R) {
                float dg = r[CH_G][k] - cg, db = r[CH_B][k] - cb;
                side[k] = dg * dg * wg + db * db * wb;
            } else if (CH == CH_G) {
                float dr = r[CH_R][k] - cr, db = r[CH_B][k] - cb;
                side[k] = dr * dr * wr + db * db * wb;
            } else {
                float dr = r[CH_R][k] - cr, dg = r[CH_G][k] - cg;
                side[k] = dr * dr * wr + dg * dg * wg;
            }
        }
        const float ci = CH == CH_R ? cr : (CH == CH_G ? cg : cb);
#pragma unroll
        for (int ab = 0; ab < 9; ++ab) {
            float m = 10000000.f;
            const int nr = flt[ab] ? 1 : N;
#pragma unroll
            for (int k = 0; k < N; ++k) {
                float d = rc[ab][k] - ci;
                float e = side[k] + d * d * wc;
                m = (k < nr) ? minr(m, e) : m;
            }
            mse[ab] += m * rp;
        }
    }
    float b0 = base[CH][0], b1 = base[CH][1];
#pragma unroll
    for (int ab = 0; ab < 9; ++ab)
        if (mse[ab] < best) {
            b0 = e0[ab];
            b1 = e1[ab];
            best = mse[ab];
        }
    cur[CH][0] = b0;
    cur[CH][1] = b1;
}

// ramp_fit_error for the one-wave kernels: lane i < n forms colour i's term from
// the wave's LDS colour rows, every lane sums the 16 terms in colour order from
// `row` (colours past n: +0, as the count-0 entries add)
template <int N>
__device__ __forceinline__ float ramp_fit_error_wave(const ColFW &u, const float r[3][4], bool flat, float *row)
{
    const float w0 = 0.3086f, w1 = 0.6094f, w2 = 0.0820f;
    const int nr = flat ? 1 : N;
    const int L = (int)(threadIdx.x & 63u);
    float term = 0.f;
    if (L < u.n) {
        const float cr = u.urow[L * 8 + CH_R], cg = u.urow[L * 8 + CH_G], cb = u.urow[L * 8 + CH_B];
        float best = 99999999999.f;
#pragma unroll
        for (int k = 0; k < N; ++k) {
            float d = (cr - r[CH_R][k]) * (cr - r[CH_R][k]) * w0 + (cg - r[CH_G][k]) * (cg - r[CH_G][k]) * w1 +
                      (cb - r[CH_B][k]) * (cb - r[CH_B][k]) * w2;
            best = (k < nr && d < best) ? d : best;
        }
        term = best * u.urow[L * 8 + 3];
    }
    if (L < 16) row[L] = term;
    wave_sync_lds();
    float err = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) err += row[i];
    return err;
}

template <int N, bool WAVE = false, class Col>
__device__ __forceinline__ void refine_channels(float cur[3][2], const Col &u, int steps)
{
    float base[3][2], wk[3][2], r[3][4];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        base[ch][0] = cur[ch][0];
        base[ch][1] = cur[ch][1];
    }
    const bool flat = expand_grid(wk, cur);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) chan_ramp<N>(r[ch], wk[ch]);
    float best;
    if constexpr (WAVE && LaneRows<Col>::v)
        best = ramp_fit_error_wave<N>(u, r, flat, u.urow + 128);   // the projection rows, free again
    else
        best = ramp_fit_error<N>(regs(u), r, flat);
    if (best == 0.f || !steps) return;
    const int lo = -(int)minr((float)steps, 8.f), hi = (int)minr((float)steps, 8.f);
    if constexpr (Col::kRefine3) {   // steps == 1 (the kernel's precondition)
        (void)lo;
        (void)hi;
        refine_pass3<N, CH_R>(cur, base, u, best);
        refine_pass3<N, CH_G>(cur, base, u, best);
        refine_pass3<N, CH_B>(cur, base, u, best);
    } else {
        const auto &ur = regs(u);
        refine_pass<N, CH_R, WAVE>(cur, base, ur, lo, hi, best);
        refine_pass<N, CH_G, WAVE>(cur, base, ur, lo, hi, best);
        refine_pass<N, CH_B, WAVE>(cur, base, ur, lo, hi, best);
    }
}

// Refine3D, amd_bcx_body.cpp:808-932 (b3DRefinement): the joint jitter of all
// six endpoint coordinates on the 565 grid, G outermost, then B, then R, each
// endpoint pair over [-steps, steps] (steps <= 8); the error of a ramp is
// accumulated channel by channel in the reference's association (G, + B, + R).
// Arrays past the block's colours hold count-0 entries (add +0).
template <int N, class Col>
__device__ void refine_3d(float cur[3][2], const Col &u, int steps)
{
    const float wr = 0.3086f, wg = 0.6094f, wb = 0.0820f;
    float base[3][2], in[3][2], wk[3][2], r[3][4];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch)
#pragma unroll
        for (int e = 0; e < 2; ++e) base[ch][e] = in[ch][e] = cur[ch][e];
    bool flat = expand_grid(wk, in);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) chan_ramp<N>(r[ch], wk[ch]);
    float best = ramp_fit_error<N>(u, r, flat);
    if (best == 0.f || !steps) return;
    const int lo = -(int)minr((float)steps, 8.f), hi = (int)minr((float)steps, 8.f);
    const float fg = (float)(1 << (8 - chan_bits(CH_G))), fb = (float)(1 << (8 - chan_bits(CH_B))),
                fr = (float)(1 << (8 - chan_bits(CH_R)));
    float eg[N][16], egb[N][16];
    for (int g0 = lo; g0 <= hi; ++g0) {
        in[CH_G][0] = minr(maxr(base[CH_G][0] + (float)g0 * fg, 0.f), 255.f);
        for (int g1 = lo; g1 <= hi; ++g1) {
            in[CH_G][1] = minr(maxr(base[CH_G][1] + (float)g1 * fg, 0.f), 255.f);
            expand_grid(wk, in);
            chan_ramp<N>(r[CH_G], wk[CH_G]);
#pragma unroll
            for (int i = 0; i < 16; ++i)
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    const float d = r[CH_G][k] - u.c(i, CH_G);
                    eg[k][i] = d * d * wg;
                }
            for (int b0 = lo; b0 <= hi; ++b0) {
                in[CH_B][0] = minr(maxr(base[CH_B][0] + (float)b0 * fb, 0.f), 255.f);
                for (int b1 = lo; b1 <= hi; ++b1) {
                    in[CH_B][1] = minr(maxr(base[CH_B][1] + (float)b1 * fb, 0.f), 255.f);
                    expand_grid(wk, in);
                    chan_ramp<N>(r[CH_B], wk[CH_B]);
#pragma unroll
                    for (int i = 0; i < 16; ++i)
#pragma unroll
                        for (int k = 0; k < N; ++k) {
                            const float d = r[CH_B][k] - u.c(i, CH_B);
                            egb[k][i] = eg[k][i] + d * d * wb;
                        }
                    for (int r0 = lo; r0 <= hi; ++r0) {
                        in[CH_R][0] = minr(maxr(base[CH_R][0] + (float)r0 * fr, 0.f), 255.f);
                        for (int r1 = lo; r1 <= hi; ++r1) {
                            in[CH_R][1] = minr(maxr(base[CH_R][1] + (float)r1 * fr, 0.f), 255.f);
                            flat = expand_grid(wk, in);
                            chan_ramp<N>(r[CH_R], wk[CH_R]);
                            const int nr = flat ? 1 : N;
                            float mse = 0.f;
#pragma unroll
                            for (int i = 0; i < 16; ++i) {
                                float m = 10000000.f;
#pragma unroll
                                for (int k = 0; k < N; ++k) {
                                    const float d = r[CH_R][k] - u.c(i, CH_R);
                                    const float e = egb[k][i] + d * d * wr;
                                    m = (k < nr) ? minr(m, e) : m;
                                }
                                mse += m * u.rpt(i);
                            }
                            if (mse < best) {
                                best = mse;
#pragma unroll
                                for (int ch = 0; ch < 3; ++ch) {
                                    cur[ch][0] = in[ch][0];
                                    cur[ch][1] = in[ch][1];
                                }
                            }
                        }
                    }
                }
            }
        }
    }
}

// RampSrchW, amd_bcx_body.cpp:398-435, over entries [I0, I1) continuing the
// running sum `error`.  Entries past n have prem = perr = 0 and prj = 0, so
// they add +0.  (prj - hi >= 0 is prj >= hi and del <= 0 is prj <= lo for
// IEEE floats with denormals kept.)
struct RampStep {
    float lo, hi, step, step_h, rstep;
};

template <int N>
__device__ __forceinline__ RampStep ramp_step(float lo, float hi)
{
    RampStep r;
    r.lo = lo;
    r.hi = hi;
    r.step = div_nm1<N>(hi - lo);
    r.step_h = r.step * (float)0.5;
    r.rstep = rcp_rn(r.step);
    return r;
}

template <int I0, int I1>
__device__ __forceinline__ float proj_ramp_error(float error, const float prj[16], const float perr[16],
                                                 const float prem[16], const RampStep &r)
{
#pragma unroll
    for (int i = I0; i < I1; ++i) {
        // branch-free form of: del <= 0 ? lo : prj - hi >= 0 ? hi : snapped
        const float del = prj[i] - r.lo;
        const float q = floorf((del + r.step_h) * r.rstep) * r.step + r.lo;
        const float vh = (prj[i] >= r.hi) ? r.hi : q;
        const float v = (prj[i] <= r.lo) ? r.lo : vh;
        float d = prj[i] - v;
        d *= d;
        error += prem[i] * d + perr[i];
    }
    return error;
}

// proj_ramp_error over entries [8, 8 + live): `live` (wave-uniform) counts the
// entries past 8 that some lane of the wave still has (unique colours n > i);
// the rest add +0 on every lane and are not evaluated.  (G1: a wave's largest
// n is 13-16, so 1.4 of 16 entries go; tools/bc1_cut_study.c.)
__device__ __forceinline__ float proj_ramp_error_tail(float error, const float prj[16], const float perr[16],
                                                      const float prem[16], const RampStep &r, int live)
{
#pragma unroll
    for (int i = 8; i < 16; ++i) {
        if (i - 8 >= live) break;
        error = proj_ramp_error<0, 1>(error, prj + i, perr + i, prem + i, r);
    }
    return error;
}

// FindAxis, amd_bcx_body.cpp:442-570.  The centred colours sh = blk - centre
// are recomputed where needed (bit-identical each time) instead of stored.
template <class Col>
__device__ __forceinline__ void principal_axis(float dir[3], float centre[3], bool &small, const Col &u)
{
    float crr[3] = {0, 0, 0}, var[3] = {0, 0, 0};
    dir[0] = dir[1] = dir[2] = 0.f;
    centre[0] = centre[1] = centre[2] = 0.f;
    float npts = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if (i < u.n) {
            centre[0] += u.blk(i, 0) * u.rpt(i);
            centre[1] += u.blk(i, 1) * u.rpt(i);
            centre[2] += u.blk(i, 2) * u.rpt(i);
            npts += u.rpt(i);
        }
    }
    centre[0] /= npts;
    centre[1] /= npts;
    centre[2] /= npts;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if (i < u.n) {
            float sh[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) sh[j] = u.blk(i, j) - centre[j];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                var[j] += sh[j] * sh[j] * u.rpt(i);
                crr[j] += sh[j] * sh[(j + 1) % 3] * u.rpt(i);
            }
        }
    }
    int i0 = 0, k = 0;
    float mx = 0.f;
    const float eps = npts * (2.f / 255.f) * (2.f / 255.f);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        if (var[j] >= eps)
            k++;
        else
            var[j] = 0.f;
        if (mx < var[j]) {
            mx = var[j];
            i0 = j;
        }
    }
    const float eps2 = npts * 3.f * (2.f / 255.f) * (2.f / 255.f);
    small = (var[0] < eps2) && (var[1] < eps2) && (var[2] < eps2);
    if (small) return;
    if (k == 1) {
        dir[0] = i0 == 0 ? 1.f : 0.f;
        dir[1] = i0 == 1 ? 1.f : 0.f;
        dir[2] = i0 == 2 ? 1.f : 0.f;
    } else if (k == 2) {
        const int i1 = (var[(i0 + 1) % 3] > 0.f) ? (i0 + 1) % 3 : (i0 + 2) % 3;
        const float cr = (i1 == (i0 + 1) % 3) ? crr[i0] : crr[(i0 + 2) % 3];
        const float q = cr / var[i0];
#pragma unroll
        for (int j = 0; j < 3; ++j) dir[j] = (j == i1) ? q : (j == i0 ? 1.f : 0.f);
    } else {
        float best_det = 100000.f;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float det = var[j] * var[(j + 1) % 3] - crr[j] * crr[j];
            if (best_det < det) {
                best_det = det;
                i0 = j;
            }
        }
        const float a = var[(i0 + 1) % 3], b = -crr[i0], c = var[i0];
        const float u0 = crr[(i0 + 2) % 3], u1 = crr[(i0 + 1) % 3];
        float s0 = a * u0 + b * u1;
        float s1 = b * u0 + c * u1;
        s0 /= best_det;
        s1 /= best_det;
#pragma unroll
        for (int j = 0; j < 3; ++j) dir[j] = (j == (i0 + 2) % 3) ? s0 + s1 : 1.f;
    }
    float len = dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2];
    len = sqrtf(len);
#pragma unroll
    for (int j = 0; j < 3; ++j) dir[j] = (len > 0.f) ? dir[j] / len : 0.f;
}

template <class Col>
__device__ __forceinline__ float last_colour(const Col &u, int j)
{
    float v = u.c(0, j);
#pragma unroll
    for (int k = 1; k < 16; ++k) v = (u.n - 1 == k) ? u.c(k, j) : v;
    return v;
}

// CompressRGBBlockX, amd_bcx_body.cpp:937-1203
template <int N, bool R3D, bool WAVE = false, class Col>
__device__ __forceinline__ void fit_endpoints(float result[3][2], const Col &u, int steps)
{
    static_assert(!(WAVE && R3D), "the wave searches cover Refine, not Refine3D");
    float rc[3][2];
    bool done = false;
    if (u.n <= 2) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            rc[j][0] = u.c(0, j);
            rc[j][1] = last_colour(u, j);
        }
        done = true;
    }
    float mid[3], dir[3];
    if (!done) {
        bool small = true;
        principal_axis(dir, mid, small, u);
        if (small) {
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                rc[j][0] = u.c(0, j);
                rc[j][1] = last_colour(u, j);
            }
            done = true;
        }
    }
    if (!done) {
        float err_g = 10000000.f;
        float dir_g[3] = {0, 0, 0}, pos_g[2] = {0, 0};
        float prj[16], perr[16], prem[16];
        for (;;) {
            float bnd0 = 1000.f, bnd1 = -1000.f;
            if constexpr (WAVE && LaneRows<Col>::v) {
                // one-wave kernels: lane i < n projects colour i (the same float
                // expressions), the wave reads the 32 results back, the bounds
                // scan runs in colour order as below
                const int L = (int)(threadIdx.x & 63u);
                float *x = u.urow + 128;
                if (L < u.n) {
                    float sh[3];
#pragma unroll
                    for (int j = 0; j < 3; ++j) sh[j] = u.urow[L * 8 + 4 + j] - mid[j];
                    const float q = sh[0] * dir[0] + sh[1] * dir[1] + sh[2] * dir[2];
                    const float e = (sh[0] - dir[0] * q) * (sh[0] - dir[0] * q) +
                                    (sh[1] - dir[1] * q) * (sh[1] - dir[1] * q) +
                                    (sh[2] - dir[2] * q) * (sh[2] - dir[2] * q);
                    x[L] = q;
                    x[16 + L] = e;
                }
                wave_sync_lds();
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const bool in = i < u.n;
                    prj[i] = in ? x[i] : 0.f;
                    perr[i] = in ? x[16 + i] : 0.f;
                    if (in) {
                        bnd0 = minr(bnd0, prj[i]);
                        bnd1 = maxr(bnd1, prj[i]);
                    }
                }
            } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                float sh[3];
#pragma unroll
                for (int j = 0; j < 3; ++j) sh[j] = u.blk(i, j) - mid[j];
                const float q = sh[0] * dir[0] + sh[1] * dir[1] + sh[2] * dir[2];
                const float e = (sh[0] - dir[0] * q) * (sh[0] - dir[0] * q) +
                                (sh[1] - dir[1] * q) * (sh[1] - dir[1] * q) +
                                (sh[2] - dir[2] * q) * (sh[2] - dir[2] * q);
                prj[i] = q;
                perr[i] = i < u.n ? e : 0.f;
                if (i < u.n) {
                    bnd0 = minr(bnd0, q);
                    bnd1 = maxr(bnd1, q);
                }
            }
            }
            const float scl0 = bnd0 - (bnd1 - bnd0) * 0.125f;
            const float scl1 = bnd1 + (bnd1 - bnd0) * 0.125f;
            const float scl2 = (scl1 - scl0) * (scl1 - scl0);
            const float over = 1.f / (scl1 - scl0);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                prj[i] = i < u.n ? (prj[i] - scl0) * over : 0.f;
                prem[i] = u.rpt(i) * scl2;   // 0 past n
            }
            bnd0 = (bnd0 - scl0) * over;
            bnd1 = (bnd1 - scl0) * over;
            const float stp = 0.025f;
            const float ls = (bnd0 - 2.f * stp > 0.f) ? bnd0 - 2.f * stp : 0.f;
            const float he = (bnd1 + 2.f * stp < 1.f) ? bnd1 + 2.f * stp : 1.f;
            // 8x8 endpoint candidates, endpoints advanced by repeated adds
            // exactly as the reference loop does (:1095-1097)
            float err = 128000.f, pos0 = 0.f, pos1 = 0.f;
            if constexpr (WAVE) {
                // candidate (l, h) on lane 8 l + h
                const int ln = (int)(threadIdx.x & 63u);
                // the loop's endpoint sequences once (the same repeated float
                // steps), picked per lane -- per-lane step loops diverge
                float lp = ls, hp = he;
                {
                    float a = ls, b = he;
#pragma unroll
                    for (int k = 1; k < 8; ++k) {
                        a += stp;
                        b -= stp;
                        lp = (ln >> 3) == k ? a : lp;
                        hp = (ln & 7) == k ? b : hp;
                    }
                }
                const RampStep rs = ramp_step<N>(lp, hp);
                float e = proj_ramp_error<8, 16>(proj_ramp_error<0, 8>(0.f, prj, perr, prem, rs), prj, perr, prem, rs);
                int o = ln;
                if (!(e < err)) {
                    e = __builtin_huge_valf();
                    o = 0x7fffffff;
                }
                wave_argmin(e, o);
                if (o != 0x7fffffff) {
                    err = e;
                    pos0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lp), o));   // o: wave-uniform
                    pos1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hp), o));
                }
            } else {
            // entries past 8 that any lane of the wave still has (uniform)
            int live = 0;
#pragma unroll
            for (int i = 8; i < 16; ++i) live += __any(u.n > i) ? 1 : 0;
            float lp = ls;
            for (int l = 0; l < 8; ++l, lp += stp) {
                float hp = he;
                for (int h = 0; h < 8; ++h, hp -= stp) {
                    // the terms are non-negative: once every block of the wave
                    // has reached its best error after 8 entries, the rest
                    // cannot make this candidate win (RampSrchW's own early out)
                    const RampStep rs = ramp_step<N>(lp, hp);
                    float e = proj_ramp_error<0, 8>(0.f, prj, perr, prem, rs);
                    if (!__all(e >= err)) e = proj_ramp_error_tail(e, prj, perr, prem, rs, live);
                    if (e < err) {
                        err = e;
                        pos0 = lp;
                        pos1 = hp;
                    }
                }
            }
            }
            pos0 = pos0 * (scl1 - scl0) + scl0;
            pos1 = pos1 * (scl1 - scl0) + scl0;
            if (!((double)err + 0.001 < (double)err_g)) break;
            err_g = err;
            dir_g[0] = dir[0];
            dir_g[1] = dir[1];
            dir_g[2] = dir[2];
            pos_g[0] = pos0;
            pos_g[1] = pos1;
            const float step = div_nm1<N>(pos1 - pos0);
            const float step_h = step * (float)0.5;
            const float rstep = rcp_rn(step);
            const float over_n = 1.f / (float)(N - 1);
            const float avg = (float)(N - 1) / 2.f;
            float crs[3] = {0, 0, 0}, len = 0.f;
            if constexpr (WAVE && LaneRows<Col>::v) {
                // lane i < n forms colour i's four products, the sums run in
                // colour order over the read-back values (the same additions)
                const int L = (int)(threadIdx.x & 63u);
                float *y = u.urow + 160;
                if (L < u.n) {
                    float sh[3];
#pragma unroll
                    for (int j = 0; j < 3; ++j) sh[j] = u.urow[L * 8 + 4 + j] - mid[j];
                    const float p0 = sh[0] * dir[0] + sh[1] * dir[1] + sh[2] * dir[2];
                    float ri, del;
                    if ((del = p0 - pos0) <= 0)
                        ri = 0.f;
                    else if (p0 - pos1 >= 0)
                        ri = (float)(N - 1);
                    else
                        ri = floorf((del + step_h) * rstep);
                    ri = (ri - avg) * over_n;
                    const float pm = ri * u.urow[L * 8 + 3];
                    y[L * 4 + 0] = ri * pm;
#pragma unroll
                    for (int j = 0; j < 3; ++j) y[L * 4 + 1 + j] = sh[j] * pm;
                }
                wave_sync_lds();
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    if (i < u.n) {
                        len += y[i * 4 + 0];
#pragma unroll
                        for (int j = 0; j < 3; ++j) crs[j] += y[i * 4 + 1 + j];
                    }
                }
            } else
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if (i < u.n) {
                    float sh[3];
#pragma unroll
                    for (int j = 0; j < 3; ++j) sh[j] = u.blk(i, j) - mid[j];
                    const float p0 = sh[0] * dir[0] + sh[1] * dir[1] + sh[2] * dir[2];   // prj0[i]
                    float ri, del;
                    if ((del = p0 - pos0) <= 0)
                        ri = 0.f;
                    else if (p0 - pos1 >= 0)
                        ri = (float)(N - 1);
                    else
                        ri = floorf((del + step_h) * rstep);
                    ri = (ri - avg) * over_n;
                    const float pm = ri * u.rpt(i);
                    len += ri * pm;
#pragma unroll
                    for (int j = 0; j < 3; ++j) crs[j] += sh[j] * pm;
                }
            }
            dir[0] = dir[1] = dir[2] = 0.f;
            if (len > 0.f) {
                dir[0] = crs[0] / len;
                dir[1] = crs[1] / len;
                dir[2] = crs[2] / len;
                float l2 = dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2];
                l2 = sqrtf(l2);
                dir[0] /= l2;
                dir[1] /= l2;
                dir[2] /= l2;
            }
        }
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int j = 0; j < 3; ++j) rc[j][k] = (pos_g[k] * dir_g[j] + mid[j]) * 255.f;
    }
    snap_grid(result, rc);
    if (R3D)
        refine_3d<N>(result, regs(u), steps);
    else
        refine_channels<N, WAVE>(result, u, steps);
}

// Leaders and ranks of the kept texels' colour keys: a kept texel leads its
// colour group if no earlier kept texel has the same key; its unique index is
// the number of leaders with a smaller key (QSortFloatCmp order,
// amd_bcx_body.cpp:103-117, dedupe :1242-1262).
__device__ __forceinline__ void rank_keys(const uint32_t key[16], bool lead[16], int ui[16], int cnt[16])
{
    // key: 24-bit colour key of a kept texel, 0xffffffff for a dropped one
    // (never equal to or below a kept key)
    int rank[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        int less = 0, same_before = 0, same = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            same += key[j] == key[i] ? 1 : 0;
            if (j < i) same_before += key[j] == key[i] ? 1 : 0;
            less += key[j] < key[i] ? 1 : 0;
        }
        lead[i] = key[i] != 0xffffffffu && same_before == 0;
        cnt[i] = same;
        rank[i] = lead[i] ? less : 0x7fff;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        int k = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) k += rank[j] < rank[i] ? 1 : 0;
        ui[i] = k;
    }
}

// 8-bit source: px[i] = R | G << 8 | B << 16 | A << 24.  thr_keep is the
// smallest alpha byte a with a / 255.0f >= alpha threshold (CompRGBABlock's
// keep test), computed on the host in the same float arithmetic.
__device__ __forceinline__ void unique_colours(ColB &u, const uint32_t px[16], bool use_alpha, uint32_t thr_keep,
                                               int &kept)
{
    uint32_t key[16];
    bool lead[16];
    int ui[16], cnt[16];
    kept = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const bool live = !use_alpha || (px[i] >> 24) >= thr_keep;
        // the float keys compare as (R, G, B) bit patterns; for v / 255.0f
        // values that is the byte order
        key[i] = live ? ((px[i] & 0xffu) << 16) | (px[i] & 0xff00u) | ((px[i] >> 16) & 0xffu) : 0xffffffffu;
        kept += live ? 1 : 0;
    }
    rank_keys(key, lead, ui, cnt);
    u.n = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) u.u[k] = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if (!lead[i]) continue;
        // colour as B, G, R bytes + count: (float)byte == (float)((double)(v / 255.0f) * 255.0)
        const uint32_t w = ((px[i] >> 16) & 0xffu) | (px[i] & 0xff00u) | ((px[i] & 0xffu) << 16) |
                           ((uint32_t)cnt[i] << 24);
#pragma unroll
        for (int k = 0; k < 16; ++k) u.u[k] = (ui[i] == k) ? w : u.u[k];
        u.n++;
    }
}

// float source (block API)
__device__ __forceinline__ void unique_colours(ColF &u, const float in[64], bool use_alpha, float thr01, int &kept)
{
    uint32_t key[16][3];
    bool live[16], lead[16];
    int rank[16], cnt[16];
    kept = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        live[i] = !use_alpha || (in[i * 4 + 3] >= thr01);
        key[i][0] = __float_as_uint(in[i * 4 + 2]);   // B
        key[i][1] = __float_as_uint(in[i * 4 + 1]);   // G
        key[i][2] = __float_as_uint(in[i * 4 + 0]);   // R
        kept += live[i] ? 1 : 0;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        int less = 0, same_before = 0, same = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (!live[j]) continue;
            const bool eq = key[j][0] == key[i][0] && key[j][1] == key[i][1] && key[j][2] == key[i][2];
            const bool lt = key[j][2] < key[i][2] ||
                            (key[j][2] == key[i][2] &&
                             (key[j][1] < key[i][1] || (key[j][1] == key[i][1] && key[j][0] < key[i][0])));
            same += eq ? 1 : 0;
            same_before += (eq && j < i) ? 1 : 0;
            less += lt ? 1 : 0;
        }
        lead[i] = live[i] && same_before == 0;
        cnt[i] = same;
        rank[i] = less;
    }
    u.n = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        u.cc[k][0] = u.cc[k][1] = u.cc[k][2] = 0.f;
        u.r[k] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if (!lead[i]) continue;
        int ui = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) ui += (lead[j] && (rank[j] < rank[i])) ? 1 : 0;
        const float cb = (float)((double)in[i * 4 + 2] * 255.0), cg = (float)((double)in[i * 4 + 1] * 255.0),
                    cr = (float)((double)in[i * 4 + 0] * 255.0);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (ui == k) {
                u.cc[k][0] = cb;
                u.cc[k][1] = cg;
                u.cc[k][2] = cr;
                u.r[k] = (float)cnt[i];
            }
        u.n++;
    }
}

// unique_colours for the one-wave block kernels: every lane holds the block (its
// 64 floats are wave-uniform), lane i < 16 ranks texel i against the others
// (16 comparisons instead of every lane running all 256), each leader stores
// its colour at its unique index in the wave's LDS rows (368 floats: colours
// 0..127, projections 128..159, products and side terms 160..223, Refine terms
// 224..367), and every lane reads the row back.  The keys, counts and ranks are the ones unique_colours
// computes, so ColF is identical.  (All lanes running the 16 x 16 comparisons on
// wave-uniform values took half of a BC1 block call: ~87 K cycles.)
__device__ __forceinline__ void unique_colours_wave(ColFW &u, const float in[64], bool use_alpha, float thr01, int &kept,
                                                    float *row)
{
    const int L = (int)(threadIdx.x & 63u);
    bool live[16];
    kept = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        live[i] = !use_alpha || (in[i * 4 + 3] >= thr01);
        kept += live[i] ? 1 : 0;
    }
    // this lane's texel (lanes >= 16: texel 15, unused)
    uint32_t k0 = 0, k1 = 0, k2 = 0;
    bool mylive = false;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        const bool me = (L == t) || (t == 15 && L > 15);
        k0 = me ? __float_as_uint(in[t * 4 + 2]) : k0;   // B
        k1 = me ? __float_as_uint(in[t * 4 + 1]) : k1;   // G
        k2 = me ? __float_as_uint(in[t * 4 + 0]) : k2;   // R
        mylive = me ? live[t] : mylive;
    }
    int less = 0, same_before = 0, same = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        if (!live[j]) continue;   // uniform
        const uint32_t j0 = __float_as_uint(in[j * 4 + 2]), j1 = __float_as_uint(in[j * 4 + 1]),
                       j2 = __float_as_uint(in[j * 4 + 0]);
        const bool eq = j0 == k0 && j1 == k1 && j2 == k2;
        const bool lt = j2 < k2 || (j2 == k2 && (j1 < k1 || (j1 == k1 && j0 < k0)));
        same += eq ? 1 : 0;
        same_before += (eq && j < L) ? 1 : 0;
        less += lt ? 1 : 0;
    }
    const bool lead = L < 16 && mylive && same_before == 0;
    const uint64_t lm = __ballot(lead);
    u.n = __popcll(lm);
    // unique index = leaders with a smaller rank (ranks of leaders are distinct)
    int ui = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int rj = __builtin_amdgcn_readlane(less, j);
        ui += (((lm >> j) & 1u) && rj < less) ? 1 : 0;
    }
    if (lead) {
        float mine[8];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float v = 0.f;
#pragma unroll
            for (int t = 0; t < 16; ++t) v = (L == t) ? in[t * 4 + 2 - c] : v;
            mine[c] = (float)((double)v * 255.0);
            mine[4 + c] = mine[c] / 255.f;   // FindAxis' input, divided by the lane that owns it
        }
        mine[3] = (float)same;
        mine[7] = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) row[ui * 8 + c] = mine[c];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const bool in_k = k < u.n;
        u.cc[k][0] = in_k ? row[k * 8 + 0] : 0.f;
        u.cc[k][1] = in_k ? row[k * 8 + 1] : 0.f;
        u.cc[k][2] = in_k ? row[k * 8 + 2] : 0.f;
        u.r[k] = in_k ? row[k * 8 + 3] : 0.f;
#pragma unroll
        for (int c = 0; c < 3; ++c) u.bk[k][c] = in_k ? row[k * 8 + 4 + c] : 0.f;
    }
    u.urow = row;
}

// Texel access for the final clustering: R, G, B as in * 255.0f and the
// alpha test !(A * 255 >= thr * 255).
struct TexB {
    const uint32_t *px;
    uint32_t thr_final;   // smallest alpha byte a with (float)a >= thr01 * 255.f
    __device__ __forceinline__ float ch(int i, int c) const { return (float)((px[i] >> (8 * c)) & 255u); }
    __device__ __forceinline__ bool transparent(int i) const { return (px[i] >> 24) < thr_final; }
    __device__ __forceinline__ const TexB &view() const { return *this; }
};
struct TexF {
    const float *in;
    float thr;   // thr01 * 255.f
    __device__ __forceinline__ float ch(int i, int c) const { return in[i * 4 + c] * 255.0f; }
    __device__ __forceinline__ bool transparent(int i) const { return !(in[i * 4 + 3] * 255.0f >= thr); }
    __device__ __forceinline__ const TexF &view() const { return *this; }
};
// One texel per lane for the one-wave kernels' final clustering (lane i < 16
// holds texel i, read from the block with a vector load, so the wave-uniform
// copy of the block need not stay live through the endpoint search)
struct TexW {
    float c[4];   // R, G, B, A as stored
    float thr;    // thr01 * 255.f
    __device__ __forceinline__ TexW(const float *__restrict__ blk, float thr_) : thr(thr_)
    {
        const int t = (int)(threadIdx.x & 15u);
#pragma unroll
        for (int k = 0; k < 4; ++k) c[k] = blk[t * 4 + k];
    }
    __device__ __forceinline__ float ch(int k) const { return c[k] * 255.0f; }
    __device__ __forceinline__ bool transparent() const { return !(c[3] * 255.0f >= thr); }
};
// The block's texels by value (TexG::view)
struct TexV {
    uint32_t px[16];
    uint32_t thr_final;
    __device__ __forceinline__ float ch(int i, int c) const { return (float)((px[i] >> (8 * c)) & 255u); }
    __device__ __forceinline__ bool transparent(int i) const { return (px[i] >> 24) < thr_final; }
};
// Texels re-read from the image when the final clustering needs them: the 16
// words are not held in VGPRs through the endpoint search (L2 hits; the
// source address is made opaque so the compiler cannot reuse the first load).
struct TexG {
    Geometry g;
    uint32_t id;   // the block; its coordinates are recomputed (one VGPR live, not three)
    bool force_alpha_one;
    uint32_t thr_final;
    __device__ __forceinline__ TexV view() const
    {
        Geometry gg = g;
        const uint8_t *src = gg.src;
        asm volatile("" : "+s"(src));
        gg.src = src;
        uint32_t slice, by, bx;
        block_coords(gg, id, slice, by, bx);
        TexV v;
        v.thr_final = thr_final;
        load_block_u8(gg, slice, by, bx, force_alpha_one, v.px);
        return v;
    }
};

// The block's texels parked in LDS (this lane's column, lane-contiguous rows
// as ColL) for the final clustering.  Re-reading them from the image (TexG)
// kept the block's 64-bit source addresses alive through the search, and the
// 3-wave build spilled those to scratch: ~64 B of scratch traffic per block.
struct TexL {
    uint32_t a;   // LDS byte address of this lane's texel 0
    uint32_t thr_final;
    __device__ __forceinline__ TexV view() const
    {
        TexV v;
        v.thr_final = thr_final;
#pragma unroll
        for (int i = 0; i < 16; ++i) v.px[i] = lds_ld_u(a, 4u * (uint32_t)(i * kLdsStride));
        return v;
    }
};

// Clstr -> ClstrBas -> ClstrIntnl, amd_bcx_body.cpp:258-378: the ramp colours
// (nr of them: 1 for a flat ramp) ...
template <int N>
__device__ __forceinline__ int final_ramp(const uint8_t ep[3][2], float r[3][4])
{
    const unsigned c0 = ((unsigned)(ep[CH_R][0] & 0xf8) << 8) | ((unsigned)(ep[CH_G][0] & 0xfc) << 3) |
                        ((unsigned)(ep[CH_B][0] & 0xf8) >> 3);
    const unsigned c1 = ((unsigned)(ep[CH_R][1] & 0xf8) << 8) | ((unsigned)(ep[CH_G][1] & 0xfc) << 3) |
                        ((unsigned)(ep[CH_B][1] & 0xf8) >> 3);
    const bool swap = (!(N & 1) && c0 <= c1) || ((N & 1) && c0 > c1);
    float ends[3][2], wk[3][2];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        ends[ch][0] = (float)ep[ch][swap ? 1 : 0];
        ends[ch][1] = (float)ep[ch][swap ? 0 : 1];
    }
    const bool flat = expand_grid(wk, ends);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) chan_ramp<N>(r[ch], wk[ch]);
    return flat ? 1 : N;
}

// ... one texel's index (N for a transparent texel) and error term (0 then)
template <int N>
__device__ __forceinline__ uint32_t final_texel(float R, float G, float B, bool transparent, const float r[3][4], int nr,
                                                float &term)
{
    const float w0 = 0.3086f, w1 = 0.6094f, w2 = 0.0820f;
    term = 0.f;
    if (transparent) return N;
    float best = 99999999999.f;
    int bi = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        if (k >= nr) break;
        const float d = (R - r[CH_R][k]) * (R - r[CH_R][k]) * w0 + (G - r[CH_G][k]) * (G - r[CH_G][k]) * w1 +
                        (B - r[CH_B][k]) * (B - r[CH_B][k]) * w2;
        if (d < best) {
            best = d;
            bi = k;
        }
    }
    term = best;
    if (bi == N - 1)
        bi = 1;
    else if (bi)
        bi++;
    return (uint32_t)bi;
}

// ... and the block's indices, the error summed in texel order
template <int N, class Tex>
__device__ __forceinline__ uint32_t final_indices(const Tex &tex, const uint8_t ep[3][2], bool use_alpha, float &err)
{
    float r[3][4];
    const int nr = final_ramp<N>(ep, r);
    uint32_t bits = 0;
    err = 0.f;
    const auto &t = tex.view();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        float term;
        const bool tr = use_alpha && t.transparent(i);
        const uint32_t idx = final_texel<N>(t.ch(i, 0), t.ch(i, 1), t.ch(i, 2), tr, r, nr, term);
        if (!tr) err += term;
        bits |= (idx & 3u) << (2 * i);
    }
    return bits;
}

// 16 bits spread to the even bits of a word
__device__ __forceinline__ uint32_t spread_even(uint32_t x)
{
    x = (x | (x << 8)) & 0x00ff00ffu;
    x = (x | (x << 4)) & 0x0f0f0f0fu;
    x = (x | (x << 2)) & 0x33333333u;
    return (x | (x << 1)) & 0x55555555u;
}

// final_indices for the one-wave kernels: lane i < 16 clusters texel i, the
// index bits come from two ballots and every lane sums the terms in texel order
// from an LDS row (16 floats; a transparent texel's +0 leaves the sum as the
// skipped addition does, the sum being >= +0 or NaN)
template <int N>
__device__ __forceinline__ uint32_t final_indices_wave(const TexW &t, const uint8_t ep[3][2], bool use_alpha, float &err,
                                                       float *row)
{
    float r[3][4];
    const int nr = final_ramp<N>(ep, r);
    const int L = (int)(threadIdx.x & 63u);
    float term;
    const uint32_t idx = final_texel<N>(t.ch(0), t.ch(1), t.ch(2), use_alpha && t.transparent(), r, nr, term);
    const uint32_t lo = (uint32_t)__ballot(L < 16 && (idx & 1u)), hi = (uint32_t)__ballot(L < 16 && (idx & 2u));
    if (L < 16) row[L] = term;
    wave_sync_lds();
    err = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) err += row[i];
    return spread_even(lo & 0xffffu) | (spread_even(hi & 0xffffu) << 1);
}

// CompRGBABlock, amd_bcx_body.cpp:1209-1297.  Returns the float error (FLT_MAX
// for a 4-colour ramp over transparent texels).
template <int N, bool R3D = false, bool WAVE = false, class Col, class Tex>
__device__ __forceinline__ float comp_rgba(const Tex &t, int steps, bool use_alpha, uint8_t ep[3][2], uint32_t &ibits,
                                           const Col &u, int kept)
{
    if (!kept) {
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            ep[ch][0] = 0;
            ep[ch][1] = 0xff;
        }
        ibits = 0xffffffffu;
        return 0.f;
    }
    if (kept != 16 && use_alpha && !(N & 1)) return 3.402823466e+38f;
    float res[3][2];
    fit_endpoints<N, R3D, WAVE>(res, u, steps);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        ep[ch][0] = (uint8_t)res[ch][0];
        ep[ch][1] = (uint8_t)res[ch][1];
    }
    float err;
    if constexpr (WAVE && LaneRows<Col>::v)
        ibits = final_indices_wave<N>(t, ep, use_alpha, err, u.urow + 128);   // the projection rows, free again
    else
        ibits = final_indices<N>(t, ep, use_alpha, err);
    return err;
}

// BC1 block words of one ramp's result: colours as 565, swapped so the block
// decodes in the 4-colour (c0 > c1) or 3-colour (c0 <= c1) mode
__device__ __forceinline__ uint2 pack_bc1(const uint8_t ep[3][2], uint32_t ibits, bool m4)
{
    const unsigned c0 = ((unsigned)(ep[CH_R][0] >> 3) << 11) | ((unsigned)(ep[CH_G][0] >> 2) << 5) |
                        (unsigned)(ep[CH_B][0] >> 3);
    const unsigned c1 = ((unsigned)(ep[CH_R][1] >> 3) << 11) | ((unsigned)(ep[CH_G][1] >> 2) << 5) |
                        (unsigned)(ep[CH_B][1] >> 3);
    uint2 out;
    if ((m4 && c0 <= c1) || (!m4 && c0 > c1))
        out.x = c1 | (c0 << 16);
    else
        out.x = c0 | (c1 << 16);
    out.y = ibits;
    return out;
}

// Image_CompressAMDBC1Block, amd_bcx_helpers.cpp:51-105.  The 3-colour result is
// packed into its block words before the 4-colour search runs, so only those two
// words and its error stay live across it.
template <bool R3D, bool WAVE = false, class Col, class Tex>
__device__ __forceinline__ uint2 encode_bc1(const Col &u, int kept, const Tex &t, int steps, bool use_alpha)
{
    uint2 b3;
    float e3f;
    {
        uint8_t ep3[3][2];
        uint32_t i3 = 0;
        e3f = comp_rgba<3, R3D, WAVE>(t, steps, use_alpha, ep3, i3, u, kept);
        b3 = pack_bc1(ep3, i3, false);
    }
    const double e3 = e3f;
    if (e3 == 0.0) return b3;
    uint8_t ep4[3][2];
    uint32_t i4 = 0;
    const double e4 = comp_rgba<4, R3D, WAVE>(t, steps, use_alpha, ep4, i4, u, kept);
    const bool m4 = !(e3 <= e4);
    return m4 ? pack_bc1(ep4, i4, true) : b3;
}

template <bool R3D>
__device__ __forceinline__ uint2 encode_bc1_u8(const uint32_t px[16], int steps, bool use_alpha, uint32_t thr_keep,
                                               const TexG &t, uint32_t lut)
{
    ColB u;
    u.lut = lut;
    int kept;
    unique_colours(u, px, use_alpha, thr_keep, kept);
    return encode_bc1<R3D>(u, kept, t, steps, use_alpha);
}

// the same with the colour words parked in LDS (ColL; w = this lane's column)
// unique_colours with each leader's word stored straight to its LDS row (row
// = its rank, w = this lane's column) instead of selected into 16 registers
// first, the word parts formed at the store (the BC1 kernel: 150 -> 120
// VGPRs, 4 waves/SIMD -- the LDS limit -- 8K G1 9.54 -> 9.17 ms, same blocks).
// Returns the number of unique colours.
__device__ __forceinline__ int unique_colours_lds(const uint32_t px[16], bool use_alpha, uint32_t thr_keep, uint32_t w,
                                                  int &kept)
{
    uint32_t key[16];
    bool lead[16];
    int ui[16], cnt[16];
    kept = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const bool live = !use_alpha || (px[i] >> 24) >= thr_keep;
        key[i] = live ? ((px[i] & 0xffu) << 16) | (px[i] & 0xff00u) | ((px[i] >> 16) & 0xffu) : 0xffffffffu;
        kept += live ? 1 : 0;
    }
    rank_keys(key, lead, ui, cnt);
    int n = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) lds_st_u(w + 4u * (uint32_t)(i * kLdsStride), 0u);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if (!lead[i]) continue;
        uint32_t c = px[i];
        asm volatile("" : "+v"(c));   // the word's parts formed here, not hoisted and held
        const uint32_t word = ((c >> 16) & 0xffu) | (c & 0xff00u) | ((c & 0xffu) << 16) | ((uint32_t)cnt[i] << 24);
        lds_st_u(w + 4u * (uint32_t)kLdsStride * (uint32_t)ui[i], word);
        n++;
    }
    return n;
}

template <bool R3D, bool S1, class Tex>
__device__ __forceinline__ uint2 encode_bc1_u8_lds(const uint32_t px[16], int steps, bool use_alpha, uint32_t thr_keep,
                                                   const Tex &t, uint32_t lut, uint32_t w)
{
    int kept;
    ColLT<S1> ul;
    ul.n = unique_colours_lds(px, use_alpha, thr_keep, w, kept);
    ul.w = w;
    ul.lut = lut;
    return encode_bc1<R3D>(ul, kept, t, steps, use_alpha);
}

template <bool R3D, bool WAVE = false>
__device__ __forceinline__ uint2 encode_bc1_f32(const float in[64], int steps, float thr01)
{
    const bool use_alpha = thr01 > 0.0f;
    ColF u;
    int kept;
    unique_colours(u, in, use_alpha, thr01, kept);
    const TexF t{in, thr01 * 255.f};
    return encode_bc1<R3D, WAVE>(u, kept, t, steps, use_alpha);
}

// --------------------------------------------------------- BC2 / BC3 ---

// Image_CompressAMDRGBSingleModeBlock (amd_bcx_helpers.cpp:142-181), the colour
// half of BC2 and BC3.  The reference's CompRGBBlock (amd_bcx_body.cpp:1299-1365)
// is undefined behaviour: its final clustering reads the 48-float RGB input with
// a stride of 4 (to index 62) and writes a 48-float buffer the same way, and it
// fits endpoints in R,G,B order but clusters in B,G,R order -- its output depends
// on stack contents.  This is its well-defined intent, the
// reference's own 4-colour CompRGBABlock fit with alpha ignored (the BC1 path's
// second candidate, amd_bcx_helpers.cpp:77-88), packed with c0 > c1 as
// :164-171 (BC2/BC3 colour blocks are always 4-colour).
template <bool R3D, bool WAVE = false, class Col, class Tex>
__device__ __forceinline__ uint2 encode_rgb4(const Col &u, int kept, const Tex &t, int steps)
{
    uint8_t ep[3][2];
    uint32_t ib = 0;
    comp_rgba<4, R3D, WAVE>(t, steps, false, ep, ib, u, kept);
    const unsigned c0 = ((unsigned)(ep[CH_R][0] >> 3) << 11) | ((unsigned)(ep[CH_G][0] >> 2) << 5) |
                        (unsigned)(ep[CH_B][0] >> 3);
    const unsigned c1 = ((unsigned)(ep[CH_R][1] >> 3) << 11) | ((unsigned)(ep[CH_G][1] >> 2) << 5) |
                        (unsigned)(ep[CH_B][1] >> 3);
    uint2 out;
    out.x = c0 <= c1 ? (c1 | (c0 << 16)) : (c0 | (c1 << 16));
    out.y = ib;
    return out;
}

// Image_CompressAMDExplictAlphaSingleModeBlock (amd_bcx_helpers.cpp:107-123): a
// = (uint8_t)(alpha * 255.0f), 4 bits per texel rounded as the reference does.
// For a byte source alpha * 255.0f == the byte; float inputs are clamped to
// [0, 255] before the conversion (out-of-range is undefined in the reference).
__device__ __forceinline__ uint32_t explicit_alpha4(uint32_t a)
{
    a = (a + ((a >> 4) < 0x8 ? 7u : 8u) - (a >> 4)) >> 4;
    return a > 0xfu ? 0xfu : a;
}

__device__ __forceinline__ uint2 encode_explicit_alpha_u8(const uint32_t px[16])
{
    uint2 out{0u, 0u};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t a = explicit_alpha4(px[i] >> 24);
        if (i < 8)
            out.x |= a << (4 * i);
        else
            out.y |= a << (4 * (i - 8));
    }
    return out;
}

__device__ __forceinline__ uint2 encode_explicit_alpha_f32(const float v[16])
{
    uint2 out{0u, 0u};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        float f = v[i] * 255.0f;
        f = f < 0.f ? 0.f : (f > 255.f ? 255.f : f);
        const uint32_t a = explicit_alpha4((uint32_t)f);
        if (i < 8)
            out.x |= a << (4 * i);
        else
            out.y |= a << (4 * (i - 8));
    }
    return out;
}

// ------------------------------------------------------------- BC4 ---

// Storage of CompBlock1's compacted value / repeat arrays (uv, ur), written at
// a running (data-dependent) position.  Private arrays indexed that way live
// in scratch; the image kernels give each lane a column of LDS instead
// (element k of lane t at k * 256 + t: consecutive lanes, consecutive banks).
struct PrivArr {
    float a[16];
    __device__ __forceinline__ float &operator[](int k) { return a[k]; }
    __device__ __forceinline__ float operator[](int k) const { return a[k]; }
};
struct LdsArr {
    float *p;   // this lane's element 0
    __device__ __forceinline__ float &operator[](int k) const { return p[k * 256]; }
};
// repeat counts (1..16) as bytes: a lane's 16 uv floats + 16 ur bytes = 80 B of LDS
// (STRIDE: bytes between a lane's counts; 1024 puts count k in byte 0 of the
// lane's own word k of a 256-lane word array)
template <int STRIDE = 256>
struct LdsCountT {
    uint8_t *p;
    struct Ref {
        uint8_t *q;
        __device__ __forceinline__ operator float() const { return (float)*q; }
        __device__ __forceinline__ Ref &operator=(float x) { *q = (uint8_t)x; return *this; }
        __device__ __forceinline__ Ref &operator+=(float x) { *q = (uint8_t)((float)*q + x); return *this; }
    };
    __device__ __forceinline__ Ref operator[](int k) const { return Ref{p + k * STRIDE}; }
};
using LdsCount = LdsCountT<256>;
struct Bc4Scratch {
    PrivArr uv, ur;
};
struct Bc4Lds {
    LdsArr uv;
    LdsCount ur;
};
struct Bc4LdsW {   // counts in the lanes' own words (the BC3 kernel borrows its texel array)
    LdsArr uv;
    LdsCountT<1024> ur;
};

// RmpSrch1 evaluated in full, amd_bcx_body.cpp:1510-1548
template <int N, class A, class C>
__device__ __forceinline__ float scalar_ramp_error(const A &v, const C &rpt, float lo, float hi, int nv)
{
    float error = 0;
    const float step = (hi - lo) / (float)(N - 1);
    const float step_h = step * 0.5f;
    const float rstep = 1.0f / step;
    for (int i = 0; i < nv; ++i) {
        float q, del;
        if ((del = v[i] - lo) <= 0)
            q = lo;
        else if (v[i] - hi >= 0)
            q = hi;
        else
            q = (floorf((del + step_h) * rstep) * step) + lo;
        const float d = v[i] - q;
        error += d * d * (float)rpt[i];
    }
    return error;
}

// CompBlock1 (8-bit integer grid), amd_bcx_body.cpp:1633-1832
template <int N, bool FIXED, class W>
__device__ void scalar_endpoints(float ramp[2], const float vals_sorted[16], W &wk)
{
    auto &uv = wk.uv;
    auto &ur = wk.ur;
    int nu = 0;
    bool need = true;
    float prev = -2.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const float x = vals_sorted[i];
        if (FIXED) {
            if (prev != x) {
                prev = x;
                if (!((double)prev <= 1.5 / 255.) && !((double)prev >= 253.5 / 255.)) {
                    uv[nu] = x;
                    ur[nu] = 1.f;
                    nu++;
                }
            } else if (nu > 0 && uv[nu - 1] == prev) {
                ur[nu - 1] += 1.f;
            }
        } else {
            if (prev != x) {
                uv[nu] = prev = x;
                ur[nu] = 1.f;
                nu++;
            } else {
                ur[nu - 1] += 1.f;
            }
        }
    }
    if (nu <= 2) {
        if (FIXED && nu == 0) {
            ramp[0] = 128.f;
            ramp[1] = ramp[0] + 1.f;
        } else {
            ramp[0] = floorf(uv[0] * 255.f + 0.5f);
            ramp[1] = (nu == 1) ? ramp[0] + 1.f : floorf(uv[1] * 255.f + 0.5f);
        }
        need = false;
    }
    if (need) {
        float lo = uv[0], hi = uv[nu - 1];
        float lr = lo, hr = hi, gl = 0, gr = 0;
        const float cntr = (lr + hr) / 2;
        float gerr = 128000.f;
        if (!(hi - lo <= 48.f / 256.f)) {
            const float llb = (0.f > lr - 0.1f) ? 0.f : lr - 0.1f;
            const float rrb = (1.f < hr + 0.1f) ? 1.f : hr + 0.1f;
            const float lrb = (cntr < lr + 0.1f) ? cntr : lr + 0.1f;
            const float rlb = (cntr > hr - 0.1f) ? cntr : hr - 0.1f;
            for (float sl = llb; sl < lrb; sl += 0.018f)
                for (float sr = rrb; rlb <= sr; sr -= 0.018f) {
                    const float e = scalar_ramp_error<N>(uv, ur, sl, sr, nu);
                    if (e < gerr) {
                        gerr = e;
                        gl = sl;
                        gr = sr;
                    }
                }
            lr = gl;
            hr = gr;
        }
        // Refine1 hill climb, amd_bcx_body.cpp:1555-1607
        const float mstep = 0.6f / 256.f;
        const float mv[3] = {0.f, -1.f, 1.f};
        int bm;
        do {
            float ca0 = lr, cb0 = hr;
            bm = -1;
#pragma unroll
            for (int m = 0; m < 9; ++m) {
                float ca = lr + mstep * mv[m / 3];
                float cb = hr + mstep * mv[m % 3];
                ca = maxr(ca, 0.f);
                cb = minr(cb, 1.f);
                const float e = scalar_ramp_error<N>(uv, ur, ca, cb, nu);
                if (e < gerr) {
                    gerr = e;
                    bm = m;
                    ca0 = ca;
                    cb0 = cb;
                }
            }
            if (bm != -1) {
                lr = ca0;
                hr = cb0;
            }
        } while (bm != -1);
        lo = lr * 255.f;
        hi = hr * 255.f;
        ramp[1] = floorf(hi + 0.5f);
        ramp[0] = floorf(lo + 0.5f);
    }
    if (ramp[0] == ramp[1]) {
        if (ramp[1] < 255.f)
            ramp[1]++;
        else
            ramp[1]--;
    }
}

// GetRmp1 + BldRmp1 + Clstr1, amd_bcx_body.cpp:1395-1505 (endpoint swap kept)
template <int N, bool FIXED>
__device__ float scalar_cluster(const float v[16], float ramp[2], uint64_t &ibits)
{
    ibits = 0;
    float err = 0.f;
    if (ramp[0] == ramp[1]) return err;
    if ((!FIXED && ramp[0] <= ramp[1]) || (FIXED && ramp[0] > ramp[1])) {
        const float t = ramp[0];
        ramp[0] = ramp[1];
        ramp[1] = t;
    }
    constexpr int NP = FIXED ? N + 2 : N;
    float pts[NP];
    pts[0] = ramp[0];
    pts[1] = ramp[1];
#pragma unroll
    for (int e = 1; e < N - 1; ++e)
        pts[e + 1] = (pts[0] * (float)(N - 1 - e) + pts[1] * (float)e) / (float)(N - 1);
    if (FIXED) {
        pts[N] = 0.f;
        pts[N + 1] = 255.f;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) pts[i] = floorf(pts[i] + 0.5f) / 1.f;
    const float over = 1.f / ((float)(1 << 8) - 1.f);
#pragma unroll
    for (int i = 0; i < NP; ++i) pts[i] *= over;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        float best = 10000000.f;
        int bi = 0;
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            float d = v[i] - pts[j];
            d *= d;
            if (d < best) {
                best = d;
                bi = j;
            }
        }
        err += best;
        ibits |= (uint64_t)bi << (3 * i);
    }
    return err;
}

template <int N, bool FIXED, class W>
__device__ float scalar_block(const float v[16], const float sorted[16], uint8_t ep[2], uint64_t &ibits, W &wk)
{
    float ramp[2];
    scalar_endpoints<N, FIXED>(ramp, sorted, wk);
    const float err = scalar_cluster<N, FIXED>(v, ramp, ibits);
    ep[0] = (uint8_t)ramp[0];
    ep[1] = (uint8_t)ramp[1];
    return err;
}

// Image_CompressAMDAlphaSingleModeBlock + EncodeAlphaBlock,
// amd_bcx_helpers.cpp:32-46, :125-140
// ascending sort by rank, as encode_bc4 (the lane version keeps its own copy inline:
// through a helper the image kernel's sort went to scratch)
__device__ __forceinline__ void bc4_sort(const float v[16], float s[16])
{
    bool nan = false;
#pragma unroll
    for (int i = 0; i < 16; ++i) nan = nan || v[i] != v[i];
    if (!nan) {
        // ranks first, then each slot gathers its texel through a select chain
        // (a scatter s[r] = v[i] became a dynamically indexed scratch store)
        int r[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            r[i] = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) r[i] += (v[j] < v[i] || (v[j] == v[i] && j < i)) ? 1 : 0;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            float x = v[0];
#pragma unroll
            for (int i = 0; i < 16; ++i) x = (r[i] == k) ? v[i] : x;
            s[k] = x;
        }
    } else {
        // A NaN texel (float sources only): QSortFCmp (:1609-1618) calls a NaN
        // equal to everything, which is no total order, so the reference's
        // qsort result is undefined (C11 7.22.5p4) and ranks would leave holes.
        // The order is the oracle's insertion sort's (orc_bcx.c
        // scalar_endpoints): each value moves left past larger ones only, as
        // a static chain of selects.
#pragma unroll
        for (int i = 0; i < 16; ++i) s[i] = v[i];
#pragma unroll
        for (int i = 1; i < 16; ++i) {
            const float t = s[i];
            bool go = true;
#pragma unroll
            for (int j = i - 1; j >= 0; --j) {
                const bool mv = go && (s[j] - t) > 0.0f;
                s[j + 1] = mv ? s[j] : (go ? t : s[j + 1]);
                go = mv;
            }
            s[0] = go ? t : s[0];
        }
    }
}

// bc4_sort for the one-wave kernels: lane i < 16 ranks texel i (16 comparisons
// instead of every lane computing all 256) and stores it at its rank in the
// wave's 16-float LDS row; every lane reads the row back.  NaN blocks take the
// register sort (uniform branch).
__device__ __forceinline__ void bc4_sort_wave(const float v[16], float s[16], float *row)
{
    bool nan = false;
#pragma unroll
    for (int i = 0; i < 16; ++i) nan = nan || v[i] != v[i];
    if (nan) {
        bc4_sort(v, s);
        return;
    }
    const int L = (int)(threadIdx.x & 63u);
    float vi = v[0];
#pragma unroll
    for (int t = 1; t < 16; ++t) vi = L == t ? v[t] : vi;
    int r = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) r += (v[j] < vi || (v[j] == vi && j < L)) ? 1 : 0;
    if (L < 16) row[r] = vi;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int k = 0; k < 16; ++k) s[k] = row[k];
}

template <class W = Bc4Scratch>
__device__ uint64_t encode_bc4(const float v[16], W wk = W())
{
    // ascending sort by rank (equal values are interchangeable)
    float s[16];
    bool nan = false;
#pragma unroll
    for (int i = 0; i < 16; ++i) nan = nan || v[i] != v[i];
    if (!nan) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            int r = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) r += (v[j] < v[i] || (v[j] == v[i] && j < i)) ? 1 : 0;
            // scatter through a select chain keeps s[] in registers
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (r == k) s[k] = v[i];
        }
    } else {
        // A NaN texel (float sources only): QSortFCmp (:1609-1618) calls a NaN
        // equal to everything, which is no total order, so the reference's
        // qsort result is undefined (C11 7.22.5p4) and ranks would leave holes.
        // The order is the oracle's insertion sort's (orc_bcx.c
        // scalar_endpoints): each value moves left past larger ones only, as
        // a static chain of selects.
#pragma unroll
        for (int i = 0; i < 16; ++i) s[i] = v[i];
#pragma unroll
        for (int i = 1; i < 16; ++i) {
            const float t = s[i];
            bool go = true;
#pragma unroll
            for (int j = i - 1; j >= 0; --j) {
                const bool mv = go && (s[j] - t) > 0.0f;
                s[j + 1] = mv ? s[j] : (go ? t : s[j + 1]);
                go = mv;
            }
            s[0] = go ? t : s[0];
        }
    }
    uint8_t ep8[2], ep6[2];
    uint64_t i8, i6 = 0;
    const float e8 = scalar_block<8, false>(v, s, ep8, i8, wk);
    float e6 = 3.402823466e+38f;
    if (!(e8 == 0.f)) e6 = scalar_block<6, true>(v, s, ep6, i6, wk);
    const bool use8 = e8 <= e6;
    const uint8_t *ep = use8 ? ep8 : ep6;
    return (uint64_t)ep[0] | ((uint64_t)ep[1] << 8) | ((use8 ? i8 : i6) << 16);
}

// ---- one 64-lane wave per block (small batches: the block-level entry points)
//
// A lane-per-block BC4 search on one noisy block is ~450 us of serial work on
// one lane (RmpSrch1's grid of up to 12 x 12 ramps, then Refine1's hill climb of
// 9 ramps a step).  Here every lane of the wave holds the block; the grid's
// (sl, sr) pairs and each climb step's 9 candidates are spread over the lanes and
// the sequential choice -- the first strictly smaller error in loop order -- is
// recovered by a (error, order) minimum.  Every ramp error is the same function
// of the same floats as in scalar_endpoints, so the blocks are bit-identical.

// The block's unique values (uv) and repeat counts (ur) as register arrays:
// every lane holds the same block, so they are built with static indices --
// the round-4 version kept them in LDS and read two LDS words per entry inside
// rolled loops, which one wave cannot hide (BC4 block kernel 39 us).  Entries
// past nu hold uv = 0, ur = 0 and add +0 to every ramp error.
template <int N>
__device__ __forceinline__ float scalar_ramp_error_reg(const float uv[16], const float ur[16], float lo, float hi)
{
    float error = 0;
    const float step = (hi - lo) / (float)(N - 1);
    const float step_h = step * 0.5f;
    const float rstep = 1.0f / step;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        float q, del;
        if ((del = uv[i] - lo) <= 0)
            q = lo;
        else if (uv[i] - hi >= 0)
            q = hi;
        else
            q = (floorf((del + step_h) * rstep) * step) + lo;
        const float d = uv[i] - q;
        error += d * d * ur[i];
    }
    return error;
}

template <int N, bool FIXED>
__device__ __forceinline__ void scalar_endpoints_wave(float ramp[2], const float vals_sorted[16], float *row)
{
    // compaction, scalar_endpoints' loop restated over runs of equal sorted
    // values: a run starts where a value differs from its predecessor (from
    // -2.f before the first, as the loop's `prev`; a NaN always differs), FIXED
    // keeps a run only strictly inside (1.5/255, 253.5/255) -- one test per run,
    // as a run's texels are one value; entry k is the k-th kept run, its value
    // and length.  (A leading run equal to -2.f is dropped: the loop's
    // out-of-range ur[-1] increment, undefined in the reference.)  Lane i < 16
    // tests sorted texel i; a kept run's first lane writes its entry to the LDS
    // row (row[16 + k] value, row[32 + k] length, zeros past the last entry).
    const int ln = (int)(threadIdx.x & 63u);
    float x = vals_sorted[0], pv = -2.f;
#pragma unroll
    for (int t = 1; t < 16; ++t) {
        x = ln == t ? vals_sorted[t] : x;
        pv = ln == t ? vals_sorted[t - 1] : pv;
    }
    const bool st = ln < 16 && x != pv;
    const bool in = !FIXED || (!((double)x <= 1.5 / 255.) && !((double)x >= 253.5 / 255.));
    const uint64_t runs = __ballot(st), kruns = __ballot(st && in);
    const int nu = __popcll(kruns);
    if (ln < 16) {
        row[16 + ln] = 0.f;
        row[32 + ln] = 0.f;
    }
    if (st && in) {
        const uint64_t later = runs & ~((2ull << ln) - 1ull);
        const int next = later ? __builtin_ctzll(later) : 16;
        const int k = __popcll(kruns & ((1ull << ln) - 1ull));
        row[16 + k] = x;
        row[32 + k] = (float)(next - ln);
    }
    wave_sync_lds();
    float uv[16], ur[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        uv[k] = row[16 + k];
        ur[k] = row[32 + k];
    }
    if (nu <= 2) {
        if (FIXED && nu == 0) {
            ramp[0] = 128.f;
            ramp[1] = ramp[0] + 1.f;
        } else {
            ramp[0] = floorf(uv[0] * 255.f + 0.5f);
            ramp[1] = (nu == 1) ? ramp[0] + 1.f : floorf(uv[1] * 255.f + 0.5f);
        }
    } else {
        float lo = uv[0], hi = uv[0];
#pragma unroll
        for (int k = 1; k < 16; ++k) hi = (k == nu - 1) ? uv[k] : hi;
        float lr = lo, hr = hi;
        const float cntr = (lr + hr) / 2;
        float gerr = 128000.f;
        if (!(hi - lo <= 48.f / 256.f)) {
            const float llb = (0.f > lr - 0.1f) ? 0.f : lr - 0.1f;
            const float rrb = (1.f < hr + 0.1f) ? 1.f : hr + 0.1f;
            const float lrb = (cntr < lr + 0.1f) ? cntr : lr + 0.1f;
            const float rlb = (cntr > hr - 0.1f) ? cntr : hr - 0.1f;
            // the loops' own iteration counts (the same float steps)
            int nl = 0, nr = 0;
            for (float sl = llb; sl < lrb; sl += 0.018f) ++nl;
            for (float sr = rrb; rlb <= sr; sr -= 0.018f) ++nr;
            float be = __builtin_huge_valf();
            int bo = 0x7fffffff;
            // the loops' endpoint sequences once (the same repeated float steps;
            // at most 0.2 / 0.018 + 1 = 12 of each), picked per lane
            float SL[16], SR[16];
            SL[0] = llb;
            SR[0] = rrb;
#pragma unroll
            for (int k = 1; k < 16; ++k) {
                SL[k] = SL[k - 1] + 0.018f;
                SR[k] = SR[k - 1] - 0.018f;
            }
            for (int t = ln; t < nl * nr; t += 64) {
                const int i = t / nr, j = t - i * nr;
                float sl = SL[0], sr = SR[0];
#pragma unroll
                for (int k = 1; k < 16; ++k) {
                    sl = k == i ? SL[k] : sl;
                    sr = k == j ? SR[k] : sr;
                }
                const float e = scalar_ramp_error_reg<N>(uv, ur, sl, sr);
                if (e < 128000.f && e < be) {   // first strictly smaller, per lane in loop order
                    be = e;
                    bo = t;
                }
            }
            wave_argmin(be, bo);
            float gl = 0.f, gr = 0.f;
            if (bo != 0x7fffffff) {
                const int i = bo / nr, j = bo - i * nr;
                gl = SL[0];
                gr = SR[0];
#pragma unroll
                for (int k = 1; k < 16; ++k) {
                    gl = k == i ? SL[k] : gl;
                    gr = k == j ? SR[k] : gr;
                }
                gerr = be;
            }
            lr = gl;
            hr = gr;
        }
        // Refine1 hill climb, amd_bcx_body.cpp:1555-1607: lane m < 9 tries move m
        const float mstep = 0.6f / 256.f;
        // (mv = {0, -1, 1}: ca moves by mv[m / 3], cb by mv[m % 3])
        const int ma = ln / 3, mb = ln % 3;
        const float mva = ma == 0 ? 0.f : (ma == 1 ? -1.f : 1.f);
        const float mvb = mb == 0 ? 0.f : (mb == 1 ? -1.f : 1.f);
        for (;;) {
            float ca = lr + mstep * mva;
            float cb = hr + mstep * mvb;
            ca = maxr(ca, 0.f);
            cb = minr(cb, 1.f);
            float e = __builtin_huge_valf();
            int o = 0x7fffffff;
            if (ln < 9) {
                const float t = scalar_ramp_error_reg<N>(uv, ur, ca, cb);
                if (t < gerr) {
                    e = t;
                    o = ln;
                }
            }
            wave_argmin(e, o);
            if (o == 0x7fffffff) break;
            lr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ca), o));   // o: wave-uniform
            hr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cb), o));
            gerr = e;
        }
        lo = lr * 255.f;
        hi = hr * 255.f;
        ramp[1] = floorf(hi + 0.5f);
        ramp[0] = floorf(lo + 0.5f);
    }
    if (ramp[0] == ramp[1]) {
        if (ramp[1] < 255.f)
            ramp[1]++;
        else
            ramp[1]--;
    }
}

// scalar_cluster with texel i on lane i: the same per-texel search, then every
// lane sums the errors in texel order and packs the indices from an LDS row
// (row[48 + i] error, row[64 + i] index).
template <int N, bool FIXED>
__device__ __forceinline__ float scalar_cluster_wave(const float v[16], float ramp[2], uint64_t &ibits, float *row)
{
    ibits = 0;
    float err = 0.f;
    if (ramp[0] == ramp[1]) return err;
    if ((!FIXED && ramp[0] <= ramp[1]) || (FIXED && ramp[0] > ramp[1])) {
        const float t = ramp[0];
        ramp[0] = ramp[1];
        ramp[1] = t;
    }
    constexpr int NP = FIXED ? N + 2 : N;
    float pts[NP];
    pts[0] = ramp[0];
    pts[1] = ramp[1];
#pragma unroll
    for (int e = 1; e < N - 1; ++e)
        pts[e + 1] = (pts[0] * (float)(N - 1 - e) + pts[1] * (float)e) / (float)(N - 1);
    if (FIXED) {
        pts[N] = 0.f;
        pts[N + 1] = 255.f;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) pts[i] = floorf(pts[i] + 0.5f) / 1.f;
    const float over = 1.f / ((float)(1 << 8) - 1.f);
#pragma unroll
    for (int i = 0; i < NP; ++i) pts[i] *= over;
    const int ln = (int)(threadIdx.x & 63u);
    float vi = v[0];
#pragma unroll
    for (int t = 1; t < 16; ++t) vi = ln == t ? v[t] : vi;
    float best = 10000000.f;
    int bi = 0;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        float d = vi - pts[j];
        d *= d;
        if (d < best) {
            best = d;
            bi = j;
        }
    }
    if (ln < 16) {
        row[48 + ln] = best;
        row[64 + ln] = (float)bi;
    }
    wave_sync_lds();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        err += row[48 + i];
        ibits |= (uint64_t)(int)row[64 + i] << (3 * i);
    }
    return err;
}

// One of encode_bc4's two ramp modes with the endpoint searches spread over the
// wave (N = 8: the 8-value ramp; N = 6, FIXED: the 6-value ramp with 0 and 255);
// every lane holds v[] and gets the mode's error and block.  row: 16 floats of
// LDS, the wave's own (80 floats: the sorted values, the compacted entries and
// the cluster step's per-texel results).  The block kernels run the two modes on
// two waves at once and join them with bc4_pick.
template <int N, bool FIXED>
__device__ __forceinline__ float encode_bc4_mode_wave(const float v[16], float *row, uint64_t &block)
{
    float s[16];
    bc4_sort_wave(v, s, row);
    float ramp[2];
    scalar_endpoints_wave<N, FIXED>(ramp, s, row);
    uint64_t ib;
    const float e = scalar_cluster_wave<N, FIXED>(v, ramp, ib, row);
    // the reference's (uint8_t) of a ramp end: a conversion to int and its low
    // byte (the 8-value mode's one-value ramp 255 / 256 stores 256 as 0); the
    // bare float-to-uint8_t conversion let the compiler join the fields with an
    // add, carrying that 256 into the next byte
    const uint32_t e0 = (uint8_t)(int)ramp[0], e1 = (uint8_t)(int)ramp[1];
    block = (uint64_t)e0 | ((uint64_t)e1 << 8) | (ib << 16);
    return e;
}

// encode_bc4's choice: the 6-value mode runs only when the 8-value error is not
// 0 (e6 = FLT_MAX otherwise), then use8 = e8 <= e6.  Computing the 6-value mode
// unconditionally and choosing this way returns the same block.
__device__ __forceinline__ uint64_t bc4_pick(float e8, uint64_t b8, float e6, uint64_t b6)
{
    return (e8 == 0.f || e8 <= e6) ? b8 : b6;
}

}  // namespace bcx

// ------------------------------------------------------------- kernels ---

struct Bc1Params {
    float alpha_threshold;
    int steps;
    int force_alpha_one;
    uint32_t thr_keep, thr_final;   // alpha-byte forms of the two threshold tests
};

template <bool R3D, bool S1>
__global__ void __launch_bounds__(256, 3) bc1_image_kernel(Geometry g, Bc1Params p, uint2 *__restrict__ dst)
{
    __shared__ float lut[256];   // byte -> v / 255.0f
    __shared__ uint32_t cols[16 * bcx::kLdsStride];   // ColL words of the workgroup's lanes
    __shared__ uint32_t texs[16 * bcx::kLdsStride];   // and their blocks' texels (TexL)
    lut[threadIdx.x] = (float)threadIdx.x / 255.0f;
    __syncthreads();
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= g.total) return;
    uint32_t slice, by, bx;
    block_coords(g, id, slice, by, bx);
    uint32_t px[16];
    load_block_u8(g, slice, by, bx, p.force_alpha_one != 0, px);
    const uint32_t ta = bcx::lds_off(texs + threadIdx.x);
#pragma unroll
    for (int i = 0; i < 16; ++i) bcx::lds_st_u(ta + 4u * (uint32_t)(i * bcx::kLdsStride), px[i]);
    const bcx::TexL t{ta, p.thr_final};
    dst[id] = bcx::encode_bc1_u8_lds<R3D, S1>(px, p.steps, p.alpha_threshold > 0.0f, p.thr_keep, t, bcx::lds_off(lut),
                                          bcx::lds_off(cols + threadIdx.x));
}

// BC2 / BC3 (amd_bc2_compressor.cpp:36-50, amd_bc3_compressor.cpp:36-50): alpha
// half (explicit 4-bit, or the BC4 interpolated alpha of
// Image_CompressAMDAlphaSingleModeBlock) then the 4-colour RGB half, one lane
// per block.  Alpha is the source's (1.0 without an alpha channel, as
// ReadNxNSplitBlockF's forceAlphaTo1).
template <bool R3D, bool S1>
__global__ void __launch_bounds__(256, 2) bc23_image_kernel(Geometry g, int fmt, Bc1Params p, uint4 *__restrict__ dst)
{
    __shared__ float lut[256];   // byte -> v / 255.0f
    __shared__ uint32_t cols[16 * bcx::kLdsStride];   // the colour half's unique colours (ColL)
    __shared__ uint32_t texs[16 * bcx::kLdsStride];   // and the block's texels (TexL), as the BC1 kernel
    lut[threadIdx.x] = (float)threadIdx.x / 255.0f;
    __syncthreads();
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= g.total) return;
    uint32_t slice, by, bx;
    block_coords(g, id, slice, by, bx);
    uint32_t px[16];
    load_block_u8(g, slice, by, bx, p.force_alpha_one != 0, px);
    uint2 a;
    if (fmt == 3) {
        // BC3's alpha half runs first: CompBlock1's running arrays borrow this
        // lane's columns of cols (uv) and texs (repeat counts) -- as the BC4
        // kernel, instead of 132 B of scratch per lane
        const bcx::Bc4LdsW wk{{reinterpret_cast<float *>(cols) + threadIdx.x},
                              {reinterpret_cast<uint8_t *>(texs + threadIdx.x)}};
        float v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = lut[px[i] >> 24];
        const uint64_t r = bcx::encode_bc4(v, wk);
        a = make_uint2((uint32_t)r, (uint32_t)(r >> 32));
    } else {
        a = bcx::encode_explicit_alpha_u8(px);
    }
    const uint32_t ta = bcx::lds_off(texs + threadIdx.x);
#pragma unroll
    for (int i = 0; i < 16; ++i) bcx::lds_st_u(ta + 4u * (uint32_t)(i * bcx::kLdsStride), px[i]);
    const bcx::TexL t{ta, 0u};
    bcx::ColLT<S1> ul;
    int kept;
    ul.w = bcx::lds_off(cols + threadIdx.x);
    ul.n = bcx::unique_colours_lds(px, false, 0u, ul.w, kept);
    ul.lut = bcx::lds_off(lut);
    const uint2 c = bcx::encode_rgb4<R3D>(ul, kept, t, p.steps);
    dst[id] = make_uint4(a.x, a.y, c.x, c.y);
}

// BC4 (one channel) / BC5 (channels 0 and 1) over an 8-bit image: the block's
// texels as packed bytes (row loads of 4 / 8 / 16 bytes for 1 / 2 / 4
// channels), each selected byte to v / 255.0f through a 256-entry LDS table.
// (A float RGBA gather indexed by a runtime channel went to scratch: 608 bytes
// per lane.)  Budgeted for 6 waves/SIMD: without SLP vectorisation (Makefile)
// BC4 takes 67 VGPRs (7 waves) and BC5 fits 6 waves (83 -> 80 VGPRs, no spill):
// 8K BC5 0.86 -> 0.83 ms, same blocks (profiles/r05_noslp_ab.txt).  (Round 4:
// 6 / 5 waves with spills, BC4 0.261 -> 0.255, BC5 0.924 -> 0.859 ms.)  BC5's two
// halves on neighbouring lanes instead -- twice the waves, one channel each --
// ran 1.08 ms: a wave lasts as long as its slowest lane, and the channels' search
// lengths vary, so 64 (R + G) chains finish sooner than 2 x 32 max(R, G) ones.
template <int FMT>
__global__ void __launch_bounds__(256, 6) bc45_image_kernel(Geometry g, int channel, uint64_t *__restrict__ dst)
{
    __shared__ float lut[256];   // byte -> v / 255.0f
    __shared__ float wk_uv[16 * 256];     // CompBlock1's uv of each lane
    __shared__ uint8_t wk_ur[16 * 256];   // and its repeat counts
    lut[threadIdx.x] = (float)threadIdx.x / 255.0f;
    __syncthreads();
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= g.total) return;
    uint32_t slice, by, bx;
    block_coords(g, id, slice, by, bx);
    uint32_t px[16];
    load_block_u8(g, slice, by, bx, false, px);
    const bcx::Bc4Lds wk{{wk_uv + threadIdx.x}, {wk_ur + threadIdx.x}};
    float v[16];
    if (FMT == 4) {
        const uint32_t sh = 8u * (uint32_t)channel;
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = lut[(px[i] >> sh) & 255u];
        dst[id] = bcx::encode_bc4(v, wk);
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = lut[px[i] & 255u];
        const uint64_t r = bcx::encode_bc4(v, wk);
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = lut[(px[i] >> 8) & 255u];
        const uint64_t gch = bcx::encode_bc4(v, wk);
        dst[2 * (size_t)id] = r;
        dst[2 * (size_t)id + 1] = gch;
    }
}

template <bool R3D>
__global__ void __launch_bounds__(256) bc1_blocks_kernel(const float *__restrict__ blocks, uint32_t n, Bc1Params p,
                                                         uint2 *__restrict__ dst)
{
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= n) return;
    float blk[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) blk[i] = blocks[(size_t)id * 64 + i];
    dst[id] = bcx::encode_bc1_f32<R3D>(blk, p.steps, p.alpha_threshold);
}

__global__ void __launch_bounds__(256) bc4_blocks_kernel(const float *__restrict__ blocks, uint32_t n,
                                                         uint64_t *__restrict__ dst)
{
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= n) return;
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = blocks[(size_t)id * 16 + i];
    dst[id] = bcx::encode_bc4(v);
}

// Small batches (Refine only): one block per 128-thread workgroup, two waves --
// wave 0 runs the 3-colour search, wave 1 the 4-colour one (independent until
// encode_bc1's comparison, amd_bcx_helpers.cpp:51-105), each search spread over
// its wave's lanes.
__global__ void __launch_bounds__(128) bc1_blocks_wave_kernel(const float *__restrict__ blocks, uint32_t n, Bc1Params p,
                                                              uint2 *__restrict__ dst)
{
    __shared__ uint2 res[2];
    __shared__ float err[2];
    __shared__ float ucol[2][368];
    const uint32_t id = blockIdx.x;
    if (id >= n) return;
    float blk[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) blk[i] = blocks[(size_t)id * 64 + i];
    const float thr01 = p.alpha_threshold;
    const bool use_alpha = thr01 > 0.0f;
    bcx::ColFW u;
    int kept;
    bcx::unique_colours_wave(u, blk, use_alpha, thr01, kept, ucol[threadIdx.x >> 6]);
    const bcx::TexW t(blocks + (size_t)id * 64, thr01 * 255.f);
    const int w = (int)(threadIdx.x >> 6);
    uint8_t ep[3][2];
    uint32_t ib = 0;
    float e;
    uint2 b;
    if (w == 0) {
        e = bcx::comp_rgba<3, false, true>(t, p.steps, use_alpha, ep, ib, u, kept);
        b = bcx::pack_bc1(ep, ib, false);
    } else {
        e = bcx::comp_rgba<4, false, true>(t, p.steps, use_alpha, ep, ib, u, kept);
        b = bcx::pack_bc1(ep, ib, true);
    }
    if ((threadIdx.x & 63u) == 0) {
        res[w] = b;
        err[w] = e;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const double e3 = err[0], e4 = err[1];
        dst[id] = (e3 == 0.0 || e3 <= e4) ? res[0] : res[1];
    }
}

// the same for BC2 / BC3: wave 0 the colour half, wave 1 the alpha half (BC3:
// waves 1 and 2 the alpha half's 8- and 6-value ramp modes, 192 threads)
__global__ void __launch_bounds__(192) bc23_blocks_wave_kernel(const float *__restrict__ blocks, uint32_t n, int fmt,
                                                               Bc1Params p, uint4 *__restrict__ dst)
{
    __shared__ uint2 res;
    __shared__ uint64_t ares[2];
    __shared__ float aerr[2];
    __shared__ float ucol[368], arow[2][80];
    const uint32_t id = blockIdx.x;
    if (id >= n) return;
    float blk[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) blk[i] = blocks[(size_t)id * 64 + i];
    const int w = (int)(threadIdx.x >> 6);
    if (w >= 1) {
        float v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = blk[i * 4 + 3];
        uint64_t r;
        float e = 0.f;
        if (fmt == 3) {
            if (w == 1)
                e = bcx::encode_bc4_mode_wave<8, false>(v, arow[0], r);
            else
                e = bcx::encode_bc4_mode_wave<6, true>(v, arow[1], r);
        } else {
            const uint2 a = bcx::encode_explicit_alpha_f32(v);
            r = (uint64_t)a.x | ((uint64_t)a.y << 32);
        }
        if ((threadIdx.x & 63u) == 0) {
            ares[w - 1] = r;
            aerr[w - 1] = e;
        }
    } else {
        bcx::ColFW u;
        int kept;
        bcx::unique_colours_wave(u, blk, false, 0.f, kept, ucol);
        const bcx::TexW t(blocks + (size_t)id * 64, 0.f);
        const uint2 r2 = bcx::encode_rgb4<false, true>(u, kept, t, p.steps);
        if (threadIdx.x == 0) res = r2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint64_t a = fmt == 3 ? bcx::bc4_pick(aerr[0], ares[0], aerr[1], ares[1]) : ares[0];
        dst[id] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), res.x, res.y);
    }
}

// wave 0 the 8-value ramp mode, wave 1 the 6-value one (encode_bc4's two
// endpoint searches, one after the other on one wave before round 5's last change)
__global__ void __launch_bounds__(128) bc4_blocks_wave_kernel(const float *__restrict__ blocks, uint32_t n,
                                                              uint64_t *__restrict__ dst)
{
    __shared__ float srow[2][80];
    __shared__ uint64_t res[2];
    __shared__ float err[2];
    const uint32_t id = blockIdx.x;
    if (id >= n) return;
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = blocks[(size_t)id * 16 + i];
    const int w = (int)(threadIdx.x >> 6);
    uint64_t b;
    float e;
    if (w == 0)
        e = bcx::encode_bc4_mode_wave<8, false>(v, srow[0], b);
    else
        e = bcx::encode_bc4_mode_wave<6, true>(v, srow[1], b);
    if ((threadIdx.x & 63u) == 0) {
        res[w] = b;
        err[w] = e;
    }
    __syncthreads();
    if (threadIdx.x == 0) dst[id] = bcx::bc4_pick(err[0], res[0], err[1], res[1]);
}

template <bool R3D>
__global__ void __launch_bounds__(256) bc23_blocks_kernel(const float *__restrict__ blocks, uint32_t n, int fmt,
                                                          Bc1Params p, uint4 *__restrict__ dst)
{
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= n) return;
    float blk[64], v[16];
#pragma unroll
    for (int i = 0; i < 64; ++i) blk[i] = blocks[(size_t)id * 64 + i];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = blk[i * 4 + 3];
    uint2 a;
    if (fmt == 3) {
        const uint64_t r = bcx::encode_bc4(v);
        a = make_uint2((uint32_t)r, (uint32_t)(r >> 32));
    } else {
        a = bcx::encode_explicit_alpha_f32(v);
    }
    bcx::ColF u;
    int kept;
    bcx::unique_colours(u, blk, false, 0.f, kept);
    const bcx::TexF t{blk, 0.f};
    const uint2 c = bcx::encode_rgb4<R3D>(u, kept, t, p.steps);
    dst[id] = make_uint4(a.x, a.y, c.x, c.y);
}

// ------------------------------------------------- non-UNORM8 sources ---

// Gather blocks [first, first + n) of a launch geometry as RGBA float blocks
// (16 texels x 4, texel-major), the float texels Image_GetPixelAtF returns
// (ReadNxNBlockF, block_utils.cpp:7-41, with its edge clamp).  kind 1: SNORM8,
// v -> max(v / 127.0f, -1.0f); kind 2: FLOAT32 as stored.  Channels past the
// source's read 0, alpha 1 (tiny_imageformat's decode is un-vendored, SURVEY.md
// 8(c): these conversions are this library's, parity against the reference
// unpinned).  The per-texel loads are scattered; this is a format-conversion
// pass, the encoders behind it dominate.
__global__ void __launch_bounds__(256) gather_f32_kernel(Geometry g, int kind, int force_alpha_one, uint32_t first,
                                                         uint32_t n, float *__restrict__ out)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    uint32_t slice, by, bx;
    block_coords(g, first + k, slice, by, bx);
    const uint8_t *img = g.src + (size_t)slice * g.row_pitch * g.height;
    float *o = out + (size_t)k * 64;
#pragma unroll
    for (int y = 0; y < 4; ++y) {
        uint32_t sy = by * 4 + y;
        sy = sy >= g.height ? g.height - 1 : sy;
#pragma unroll
        for (int x = 0; x < 4; ++x) {
            uint32_t sx = bx * 4 + x;
            sx = sx >= g.width ? g.width - 1 : sx;
            float v[4] = {0.f, 0.f, 0.f, 1.f};
            if (kind == 1) {
                const int8_t *p = reinterpret_cast<const int8_t *>(img + (size_t)sy * g.row_pitch + (size_t)sx * g.channels);
                for (uint32_t c = 0; c < g.channels && c < 4; ++c) v[c] = maxr((float)p[c] / 127.0f, -1.0f);
            } else {
                const float *p = reinterpret_cast<const float *>(img + (size_t)sy * g.row_pitch) + (size_t)sx * g.channels;
                for (uint32_t c = 0; c < g.channels && c < 4; ++c) v[c] = p[c];
            }
            if (force_alpha_one) v[3] = 1.f;
            float *t = o + (y * 4 + x) * 4;
            t[0] = v[0];
            t[1] = v[1];
            t[2] = v[2];
            t[3] = v[3];
        }
    }
}

// BC4 (channel `channel`) or BC5 (channels 0, 1) from RGBA float blocks
__global__ void __launch_bounds__(256) bc45_rgba_blocks_kernel(const float *__restrict__ blocks, uint32_t n, int fmt,
                                                               int channel, uint64_t *__restrict__ dst)
{
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= n) return;
    float v[16];
    if (fmt == 4) {
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = blocks[(size_t)id * 64 + i * 4 + channel];
        dst[id] = bcx::encode_bc4(v);
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = blocks[(size_t)id * 64 + i * 4];
        dst[2 * (size_t)id] = bcx::encode_bc4(v);
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = blocks[(size_t)id * 64 + i * 4 + 1];
        dst[2 * (size_t)id + 1] = bcx::encode_bc4(v);
    }
}

// ------------------------------------------------------------- decode ---

namespace dec {

__device__ __forceinline__ void rgb565(uint32_t c, int v[3])
{
    const int r = (int)(c >> 11) & 31, g = (int)(c >> 5) & 63, b = (int)c & 31;
    v[0] = (r << 3) | (r >> 2);
    v[1] = (g << 2) | (g >> 4);
    v[2] = (b << 3) | (b >> 2);
}

// colour block (8 bytes) -> 16 packed RGBA words; four_only: BC2/BC3
__device__ __forceinline__ void colour_block(uint2 blk, bool four_only, uint32_t px[16])
{
    const uint32_t c0 = blk.x & 0xffffu, c1 = blk.x >> 16;
    int e0[3], e1[3];
    rgb565(c0, e0);
    rgb565(c1, e1);
    const bool four = four_only || c0 > c1;
    uint32_t pal[4];
    pal[0] = (uint32_t)e0[0] | ((uint32_t)e0[1] << 8) | ((uint32_t)e0[2] << 16) | 0xff000000u;
    pal[1] = (uint32_t)e1[0] | ((uint32_t)e1[1] << 8) | ((uint32_t)e1[2] << 16) | 0xff000000u;
    pal[2] = pal[3] = 0xff000000u;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const uint32_t v2 = four ? (uint32_t)(2 * e0[c] + e1[c] + 1) / 3 : (uint32_t)(e0[c] + e1[c] + 1) / 2;
        const uint32_t v3 = four ? (uint32_t)(e0[c] + 2 * e1[c] + 1) / 3 : 0u;
        pal[2] |= v2 << (8 * c);
        pal[3] |= v3 << (8 * c);
    }
    if (!four) pal[3] = 0u;   // transparent black
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t k = (blk.y >> (2 * i)) & 3u;
        px[i] = k == 0 ? pal[0] : (k == 1 ? pal[1] : (k == 2 ? pal[2] : pal[3]));
    }
}

// BC4 block -> 16 values
__device__ __forceinline__ void scalar_block(uint2 blk, uint32_t v[16])
{
    const int e0 = (int)(blk.x & 0xffu), e1 = (int)((blk.x >> 8) & 0xffu);
    const uint64_t bits = ((uint64_t)blk.x | ((uint64_t)blk.y << 32)) >> 16;
    const bool eight = e0 > e1;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int k = (int)((bits >> (3 * i)) & 7u);
        int r;
        if (k == 0)
            r = e0;
        else if (k == 1)
            r = e1;
        else if (eight)
            r = ((8 - k) * e0 + (k - 1) * e1 + 3) / 7;
        else
            r = k == 6 ? 0 : (k == 7 ? 255 : ((6 - k) * e0 + (k - 1) * e1 + 2) / 5);
        v[i] = (uint32_t)r;
    }
}

}  // namespace dec

// One lane per block; a block's four rows are written as 16-byte stores
// (adjacent lanes = adjacent blocks: coalesced row segments) when whole.
__global__ void __launch_bounds__(256) bcx_decode_kernel(const uint8_t *__restrict__ blocks, int fmt, uint32_t width,
                                                         uint32_t height, uint32_t bx_count, uint32_t total,
                                                         uint8_t *__restrict__ out, size_t row_pitch)
{
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= total) return;
    const uint32_t by_count = (height + 3) / 4;
    const uint32_t bx = id % bx_count, r = id / bx_count, by = r % by_count, slice = r / by_count;
    uint32_t px[16];
    if (fmt == 1) {
        dec::colour_block(reinterpret_cast<const uint2 *>(blocks)[id], false, px);
    } else if (fmt == 4) {
        uint32_t v[16];
        dec::scalar_block(reinterpret_cast<const uint2 *>(blocks)[id], v);
#pragma unroll
        for (int i = 0; i < 16; ++i) px[i] = v[i] | 0xff000000u;
    } else {
        const uint4 b = reinterpret_cast<const uint4 *>(blocks)[id];
        if (fmt == 5) {
            uint32_t v[16], w[16];
            dec::scalar_block(make_uint2(b.x, b.y), v);
            dec::scalar_block(make_uint2(b.z, b.w), w);
#pragma unroll
            for (int i = 0; i < 16; ++i) px[i] = v[i] | (w[i] << 8) | 0xff000000u;
        } else {
            dec::colour_block(make_uint2(b.z, b.w), true, px);
            if (fmt == 3) {
                uint32_t a[16];
                dec::scalar_block(make_uint2(b.x, b.y), a);
#pragma unroll
                for (int i = 0; i < 16; ++i) px[i] = (px[i] & 0x00ffffffu) | (a[i] << 24);
            } else {
                const uint64_t ab = (uint64_t)b.x | ((uint64_t)b.y << 32);
#pragma unroll
                for (int i = 0; i < 16; ++i) px[i] = (px[i] & 0x00ffffffu) | ((uint32_t)((ab >> (4 * i)) & 15u) * 17u << 24);
            }
        }
    }
    uint8_t *img = out + (size_t)slice * row_pitch * height;
    const uint32_t x0 = bx * 4, y0 = by * 4;
    const bool whole = x0 + 4 <= width && y0 + 4 <= height && ((row_pitch | (uintptr_t)out) & 15) == 0;
#pragma unroll
    for (int y = 0; y < 4; ++y) {
        if (y0 + y >= height) break;
        uint8_t *row = img + (size_t)(y0 + y) * row_pitch + (size_t)x0 * 4;
        if (whole) {
            *reinterpret_cast<uint4 *>(row) = make_uint4(px[4 * y], px[4 * y + 1], px[4 * y + 2], px[4 * y + 3]);
        } else {
#pragma unroll
            for (int x = 0; x < 4; ++x)
                if (x0 + x < width) *reinterpret_cast<uint32_t *>(row + 4 * x) = px[4 * y + x];
        }
    }
}

// ------------------------------------------------------------ launchers ---

hipError_t launch_gather_f32(const Geometry &g, int kind, int force_alpha_one, uint32_t first, uint32_t n, float *out,
                             hipStream_t s)
{
    const uint32_t wg = 256, grid = (n + wg - 1) / wg;
    hipLaunchKernelGGL(gather_f32_kernel, dim3(grid), dim3(wg), 0, s, g, kind, force_alpha_one, first, n, out);
    return hipGetLastError();
}

hipError_t launch_bc45_rgba_blocks(const float *blocks, uint32_t n, int fmt, int channel, void *dst, hipStream_t s)
{
    const uint32_t wg = 256, grid = (n + wg - 1) / wg;
    hipLaunchKernelGGL(bc45_rgba_blocks_kernel, dim3(grid), dim3(wg), 0, s, blocks, n, fmt, channel, (uint64_t *)dst);
    return hipGetLastError();
}

hipError_t launch_bcx_decode(const uint8_t *blocks, int fmt, uint32_t width, uint32_t height, uint32_t slices,
                             uint8_t *out, size_t row_pitch, hipStream_t s)
{
    const uint32_t bx = (width + 3) / 4, by = (height + 3) / 4;
    const uint64_t total = (uint64_t)bx * by * slices;
    if (total > 0xffffffffull) return hipErrorInvalidValue;
    const uint32_t wg = 256, grid = (uint32_t)((total + wg - 1) / wg);
    hipLaunchKernelGGL(bcx_decode_kernel, dim3(grid), dim3(wg), 0, s, blocks, fmt, width, height, bx, (uint32_t)total,
                       out, row_pitch);
    return hipGetLastError();
}


// smallest alpha byte passing `pass(a)` (256 if none); pass is monotone in a
template <class F>
static uint32_t first_byte(F pass)
{
    for (uint32_t a = 0; a < 256; ++a)
        if (pass(a)) return a;
    return 256;
}

hipError_t launch_bc1_image(const Geometry &g, float thr, int steps, int force_alpha_one, int r3d, void *dst,
                            hipStream_t s)
{
    // CompRGBABlock keeps a texel when a / 255.0f >= thr; ClstrIntnl marks it
    // transparent when !(a / 255.0f * 255.0f >= thr * 255.f), and a / 255.0f *
    // 255.0f == a for every byte.  Both tests are monotone in a.
    const volatile float t = thr;
    const float t255 = t * 255.f;
    const uint32_t keep = first_byte([&](uint32_t a) { return (float)a / 255.0f >= t; });
    const uint32_t fin = first_byte([&](uint32_t a) { return (float)a >= t255; });
    const Bc1Params p{thr, steps, force_alpha_one, keep, fin};
    const uint32_t wg = 256, grid = (g.total + wg - 1) / wg;
    if (r3d)
        hipLaunchKernelGGL((bc1_image_kernel<true, false>), dim3(grid), dim3(wg), 0, s, g, p, (uint2 *)dst);
    else if (steps == 1)
        hipLaunchKernelGGL((bc1_image_kernel<false, true>), dim3(grid), dim3(wg), 0, s, g, p, (uint2 *)dst);
    else
        hipLaunchKernelGGL((bc1_image_kernel<false, false>), dim3(grid), dim3(wg), 0, s, g, p, (uint2 *)dst);
    return hipGetLastError();
}

hipError_t launch_bc23_image(const Geometry &g, int fmt, int steps, int force_alpha_one, int r3d, void *dst,
                             hipStream_t s)
{
    const Bc1Params p{0.f, steps, force_alpha_one, 0u, 0u};
    const uint32_t wg = 256, grid = (g.total + wg - 1) / wg;
    if (r3d)
        hipLaunchKernelGGL((bc23_image_kernel<true, false>), dim3(grid), dim3(wg), 0, s, g, fmt, p, (uint4 *)dst);
    else if (steps == 1)
        hipLaunchKernelGGL((bc23_image_kernel<false, true>), dim3(grid), dim3(wg), 0, s, g, fmt, p, (uint4 *)dst);
    else
        hipLaunchKernelGGL((bc23_image_kernel<false, false>), dim3(grid), dim3(wg), 0, s, g, fmt, p, (uint4 *)dst);
    return hipGetLastError();
}

// Below this many blocks a wave per block (the *_wave_kernel launches) finishes
// sooner than a lane per block: the batch cannot fill the chip lane-wise, and a
// block's serial search is the call's latency.
constexpr uint32_t kWaveBlocks = 4096;

hipError_t launch_bc23_blocks(const float *blocks, uint32_t n, int fmt, int steps, int r3d, void *dst, hipStream_t s)
{
    const Bc1Params p{0.f, steps, 0, 0u, 0u};
    if (n < kWaveBlocks && !r3d) {
        hipLaunchKernelGGL(bc23_blocks_wave_kernel, dim3(n), dim3(fmt == 3 ? 192 : 128), 0, s, blocks, n, fmt, p,
                           (uint4 *)dst);
        return hipGetLastError();
    }
    const uint32_t wg = 256, grid = (n + wg - 1) / wg;
    if (r3d)
        hipLaunchKernelGGL(bc23_blocks_kernel<true>, dim3(grid), dim3(wg), 0, s, blocks, n, fmt, p, (uint4 *)dst);
    else
        hipLaunchKernelGGL(bc23_blocks_kernel<false>, dim3(grid), dim3(wg), 0, s, blocks, n, fmt, p, (uint4 *)dst);
    return hipGetLastError();
}

hipError_t launch_bc45_image(const Geometry &g, int fmt, int channel, void *dst, hipStream_t s)
{
    const uint32_t wg = 256, grid = (g.total + wg - 1) / wg;
    if (fmt == 4)
        hipLaunchKernelGGL(bc45_image_kernel<4>, dim3(grid), dim3(wg), 0, s, g, channel, (uint64_t *)dst);
    else
        hipLaunchKernelGGL(bc45_image_kernel<5>, dim3(grid), dim3(wg), 0, s, g, channel, (uint64_t *)dst);
    return hipGetLastError();
}

hipError_t launch_bc1_blocks(const float *blocks, uint32_t n, float thr, int steps, int r3d, void *dst, hipStream_t s)
{
    const Bc1Params p{thr, steps, 0, 0u, 0u};
    if (n < kWaveBlocks && !r3d) {
        hipLaunchKernelGGL(bc1_blocks_wave_kernel, dim3(n), dim3(128), 0, s, blocks, n, p, (uint2 *)dst);
        return hipGetLastError();
    }
    const uint32_t wg = 256, grid = (n + wg - 1) / wg;
    if (r3d)
        hipLaunchKernelGGL(bc1_blocks_kernel<true>, dim3(grid), dim3(wg), 0, s, blocks, n, p, (uint2 *)dst);
    else
        hipLaunchKernelGGL(bc1_blocks_kernel<false>, dim3(grid), dim3(wg), 0, s, blocks, n, p, (uint2 *)dst);
    return hipGetLastError();
}

hipError_t launch_bc4_blocks(const float *blocks, uint32_t n, void *dst, hipStream_t s)
{
    if (n < kWaveBlocks) {
        hipLaunchKernelGGL(bc4_blocks_wave_kernel, dim3(n), dim3(128), 0, s, blocks, n, (uint64_t *)dst);
        return hipGetLastError();
    }
    const uint32_t wg = 256, grid = (n + wg - 1) / wg;
    hipLaunchKernelGGL(bc4_blocks_kernel, dim3(grid), dim3(wg), 0, s, blocks, n, (uint64_t *)dst);
    return hipGetLastError();
}

}  // namespace gic

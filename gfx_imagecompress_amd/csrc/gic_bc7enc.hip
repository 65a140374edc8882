// gic_bc7enc.hip -- bc7enc16, the reference's fast BC7 encoder
// (src/richgel999_bc7enc16.cpp, reached from ImageCompress_Compress(DXBC7,
// fast = true), imagecompress.cpp:34-36), for CDNA4.
//
// Mapping: one lane per 4x4 block.  bc7enc16 is a short, branchy per-block
// search (mode 6 over the whole block, then mode 1 on the one partition its
// estimator picks), with no search breadth that would feed a whole wave per
// block, so the 16 texels live in 16 VGPRs as packed RGBA8 words and every
// step is lane-local.  Subsets are 16-bit texel masks walked in texel order,
// so each float sum adds the same texels in the same order as the reference's
// compacted lists (bit-exact under the numerics flags of gic_common.h).
// Selectors are 4-bit nibbles of a 64-bit word.  The least-squares selector
// weights and the single-colour table sit in LDS.
//
// Error arithmetic is 32-bit: the largest per-texel error (perceptual RGBA:
// 512*510^2 + 103*803^2 + 18*946^2 + 128*255^2 < 2.3e8) times 16 texels stays
// below 2^32, so the reference's uint64 totals never exceed 32 bits and
// 0xffffffff can stand for its UINT64_MAX "no solution yet".
#include <type_traits>

#include "bc7_tables.h"
#include "bc7enc_tables.h"
#include "gic_common.h"

namespace gic {
namespace {

constexpr uint32_t kNone = 0xffffffffu;

struct EncCfg {                 // bc7enc16_compress_block_params (richgel999_bc7enc16.h:17-36)
    uint32_t uber;              // m_uber_level 0..4
    uint32_t max_parts;         // m_max_partitions_mode1 0..64
    uint32_t lsq;               // m_try_least_squares
    uint32_t filterbank;        // m_mode1_partition_estimation_filterbank
    uint32_t w[4];              // error weights after bc7enc16_compress_block's scaling (:1524-1535)
};

struct EncLds {
    float wx[96];               // g_bc7_weights3x (0..31), g_bc7_weights4x (32..95)
    uint32_t one[512];          // g_bc7_mode_1_optimal_endpoints
};

__device__ __forceinline__ uint32_t ch(uint32_t c, int k) { return (c >> (8 * k)) & 0xffu; }
__device__ __forceinline__ float clampf_r(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ float sat(float v) { return clampf_r(v, 0.f, 1.0f); }
__device__ __forceinline__ int clampi_r(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ uint32_t sel_at(uint64_t s, int i) { return (uint32_t)(s >> (4 * i)) & 15u; }


// g_bc7_weights3/4 (:130-131): round(64 s / (N - 1))
__device__ __forceinline__ uint32_t bc7w(uint32_t s, uint32_t N)
{
    return N == 16 ? (s * 64u + 7u) / 15u : (s * 64u + 3u) / 7u;
}

// 24-bit multiplies (full rate).  Every factor below is a channel difference
// |d| <= 946 or a weight times one (<= 512 * 946 < 2^23), and every product and
// sum stays below 2^31, so these equal the reference's uint32 arithmetic.
__device__ __forceinline__ int mul24(int a, int b) { return __mul24(a, b); }
__device__ __forceinline__ int mad24(int a, int b, int c) { return __mul24(a, b) + c; }

// interpolated channel k of the ramp point with weight w (:445, :1053)
__device__ __forceinline__ int lerp_ch(uint32_t a, uint32_t b, int k, uint32_t w)
{
    return (int)((ch(a, k) * (64u - w) + ch(b, k) * w + 32u) >> 6);
}

struct Prob {           // one subset problem (color_cell_compressor_params :282-295)
    uint32_t mask;      // texels of the subset
    uint32_t n;         // its texel count
    uint32_t nsel;      // 16 (mode 6) / 8 (mode 1)
    uint32_t cbits;     // 7 / 6
    bool mode1;         // shared p-bit, single-colour paths, degenerate-endpoint fix
    bool alpha;         // RGBA (mode 6 of a block with alpha)
};

struct Res {            // color_cell_compressor_results :297-305
    uint32_t err;
    uint32_t lo, hi;    // quantised endpoints, channel k in byte k
    uint32_t pb0, pb1;
    uint64_t sel;       // selector of texel i in nibble i (texels of the subset only)
};

// The block's texels live in the workgroup's LDS, not in registers: with the
// 16 texel words held through the whole search the lane kernels spilled ~100
// VGPRs at 3 waves/SIMD (8x the algorithmic HBM bytes in scratch traffic,
// round 5).  Each lane owns a column of rows (row r of lane t at word r *
// STRIDE + t, so a wave's reads are conflict-free; STRIDE = the workgroup's
// lanes: 256 for the lane-per-block kernels, 64 for the one-wave block
// kernel).  The read address is opaque at every use, so the loads stay where
// the texels are used instead of being hoisted back into registers.
//
// Perceptual metric (YccT): rows 0..15 / 16..31 / 32..47 hold the texel's
// transforms l, cr, cb (compute_color_distance_rgb, :331-339) scaled by 2^13,
// less one unit of 2^13, with the texel's bytes in the low bits:
//   L  = (l  - 1) * 2^13 + (1 | r << 1 | (a & 15) << 9)
//   CR = (cr - 1) * 2^13 + (1 | g << 1 | (a >> 4) << 9)
//   CB = (cb - 1) * 2^13 + (1 | b << 1)
// (low parts in [1, 8191]).  A ramp colour's transforms are scaled by 2^13
// exactly (ycc_ramp: the same three multiply-adds with scaled constants), so
// for a ramp point and a texel L1 - L2 = (l1 - l2) * 2^13 + d with d in
// [1, 8191]: d never carries past a multiple of 2^21, and (L1 - L2) >> 21 =
// (l1 - l2) >> 8 exactly, likewise CR and CB; every difference stays inside
// int32 (|cr1 - cr2| <= 261120, * 2^13 + 8191 < 2^31).  So the metric costs
// what it did with plain l / cr / cb rows, and the texel words need no rows of
// their own (48 rows, 48 KB per workgroup: the LDS budget of 3 workgroups per
// CU); a texel's bytes come back with one bit-field extract each.
template <uint32_t STRIDE>
struct YccT {
    uint32_t a;   // LDS byte address of this lane's row-0 word
    static constexpr uint32_t kRows = 48;
    __device__ __forceinline__ int at(int row) const
    {
        uint32_t b = a;
        asm volatile("" : "+v"(b));
        return *(const __attribute__((address_space(3))) int *)(size_t)(b + 4u * (uint32_t)row * STRIDE);
    }
    __device__ __forceinline__ int l(int i) const { return at(i); }
    __device__ __forceinline__ int cr(int i) const { return at(16 + i); }
    __device__ __forceinline__ int cb(int i) const { return at(32 + i); }
    __device__ __forceinline__ uint32_t word(int i) const
    {
        const uint32_t x = (uint32_t)l(i), y = (uint32_t)cr(i), z = (uint32_t)cb(i);
        return __builtin_amdgcn_ubfe(x, 1, 8) | __builtin_amdgcn_ubfe(y, 1, 8) << 8 | __builtin_amdgcn_ubfe(z, 1, 8) << 16 |
               __builtin_amdgcn_ubfe(x, 9, 4) << 24 | __builtin_amdgcn_ubfe(y, 9, 4) << 28;
    }
    // texel i's channels (alpha only when asked for, else 0)
    __device__ __forceinline__ void chans(int i, bool alpha, uint32_t c[4]) const
    {
        const uint32_t x = (uint32_t)l(i), y = (uint32_t)cr(i), z = (uint32_t)cb(i);
        c[0] = __builtin_amdgcn_ubfe(x, 1, 8);
        c[1] = __builtin_amdgcn_ubfe(y, 1, 8);
        c[2] = __builtin_amdgcn_ubfe(z, 1, 8);
        c[3] = alpha ? __builtin_amdgcn_ubfe(x, 9, 4) | __builtin_amdgcn_ubfe(y, 9, 4) << 4 : 0u;
    }
    __device__ __forceinline__ void put(int i, uint32_t w) const
    {
        typedef __attribute__((address_space(3))) int lds_i32;
        const int r = (int)(w & 0xffu), g = (int)((w >> 8) & 0xffu), b = (int)((w >> 16) & 0xffu);
        const int al = (int)(w >> 24);
        const int l_ = r * 109 + g * 366 + b * 37;
        const int cr_ = (r << 9) - l_, cb_ = (b << 9) - l_;
        *(lds_i32 *)(size_t)(a + 4u * (uint32_t)i * STRIDE) = (l_ - 1) * 8192 + (1 | r << 1 | (al & 15) << 9);
        *(lds_i32 *)(size_t)(a + 4u * (uint32_t)(16 + i) * STRIDE) = (cr_ - 1) * 8192 + (1 | g << 1 | (al >> 4) << 9);
        *(lds_i32 *)(size_t)(a + 4u * (uint32_t)(32 + i) * STRIDE) = (cb_ - 1) * 8192 + (1 | b << 1);
    }
};
template <uint32_t STRIDE>
struct TexT {
    uint32_t a;
    static constexpr uint32_t kRows = 16;
    __device__ __forceinline__ int at(int row) const
    {
        uint32_t b = a;
        asm volatile("" : "+v"(b));
        return *(const __attribute__((address_space(3))) int *)(size_t)(b + 4u * (uint32_t)row * STRIDE);
    }
    __device__ __forceinline__ int l(int) const { return 0; }   // (perceptual paths only)
    __device__ __forceinline__ int cr(int) const { return 0; }
    __device__ __forceinline__ int cb(int) const { return 0; }
    __device__ __forceinline__ uint32_t word(int i) const { return (uint32_t)at(i); }
    __device__ __forceinline__ void chans(int i, bool alpha, uint32_t c[4]) const
    {
        const uint32_t w = word(i);
#pragma unroll
        for (int k = 0; k < 3; ++k) c[k] = ch(w, k);
        c[3] = alpha ? ch(w, 3) : 0u;
    }
    __device__ __forceinline__ void put(int i, uint32_t w) const
    {
        *(__attribute__((address_space(3))) int *)(size_t)(a + 4u * (uint32_t)i * STRIDE) = (int)w;
    }
};
constexpr uint32_t kYccStride = 256;
using Ycc = YccT<kYccStride>;
template <bool P, uint32_t STRIDE>
using TexSrc = typename std::conditional<P, YccT<STRIDE>, TexT<STRIDE>>::type;

// a texel word of the block (from LDS, see above)
template <class Y>
__device__ __forceinline__ uint32_t tex(const Y &y, int i)
{
    return y.word(i);
}

// scale_color :307-323 (n = component bits + p-bit)
__device__ __forceinline__ uint32_t expand(uint32_t q, uint32_t n)
{
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t v = ch(q, k) << (8 - n);
        r |= ((v | (v >> n)) & 0xffu) << (8 * k);
    }
    return r;
}

// the YCbCr-style transform of compute_color_distance_rgb (:331-339) of a
// ramp colour, scaled by 2^13 (see YccT)
__device__ __forceinline__ void ycc_ramp(int r, int g, int b, int &l, int &cr, int &cb)
{
    l = r * (109 * 8192) + g * (366 * 8192) + b * (37 * 8192);
    cr = (r << 22) - l;
    cb = (b << 22) - l;
}

// weighted squared distance w0 d0^2 + w1 d1^2 + w2 d2^2 [+ e]
__device__ __forceinline__ uint32_t wsq(int d0, int d1, int d2, const EncCfg &cf, int e = 0)
{
    // |d| <= 946 and w <= 512 (see above): tell the optimiser, so that every
    // product is a 24-bit multiply without masking
    __builtin_assume((uint32_t)(d0 + 1024) < 2048u);
    __builtin_assume((uint32_t)(d1 + 1024) < 2048u);
    __builtin_assume((uint32_t)(d2 + 1024) < 2048u);
    const uint32_t s0 = (uint32_t)(d0 * d0), s1 = (uint32_t)(d1 * d1), s2 = (uint32_t)(d2 * d2);
    __builtin_assume(s0 < (1u << 20));
    __builtin_assume(s1 < (1u << 20));
    __builtin_assume(s2 < (1u << 20));
    return (uint32_t)e + __umul24(cf.w[0], s0) + __umul24(cf.w[1], s1) + __umul24(cf.w[2], s2);
}

// compute_color_distance_rgb with perceptual = true, from a ramp colour's
// packed transforms (ycc_ramp) and a texel's (YccT): (l1 - l2) >> 8 etc.
__device__ __forceinline__ uint32_t ycc_err(int l1, int cr1, int cb1, int l2, int cr2, int cb2, const EncCfg &cf,
                                            int e = 0)
{
    return wsq((l1 - l2) >> 21, (cr1 - cr2) >> 21, (cb1 - cb2) >> 21, cf, e);
}

// The search below runs K subset problems in lockstep: K = 1 is one problem on
// pr[0].mask (mode 6, the whole block), K = 2 the two subsets of a mode-1
// partition (m0 = the texels of subset 0).  Every per-texel pass scores each
// texel against its own subset's candidate, so mode 1's two subsets share
// their passes over the block.
template <int K>
__device__ __forceinline__ bool first_subset(uint32_t m0, int i)
{
    return K == 1 || ((m0 >> i) & 1u);
}

__device__ __forceinline__ uint64_t nibble_mask(uint32_t m)
{
    uint64_t r = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) r |= (uint64_t)(((m >> i) & 1u) ? 15u : 0u) << (4 * i);
    return r;
}

// evaluate_solution :405-572 for the candidates (lo, hi, pb) of the K problems;
// a problem's result is updated only if want[s] (find_optimal_solution's
// changed-endpoints test).  Texels outside a K = 1 problem's mask are computed
// and discarded (branch-free); the integer totals do not depend on order.
// bit i of m (i < 16) to bit 4i (the selector nibbles' bit 0)
__device__ __forceinline__ uint64_t spread4(uint32_t m)
{
    uint64_t x = m & 0xffffu;
    x = (x | (x << 24)) & 0x000000ff000000ffull;
    x = (x | (x << 12)) & 0x000f000f000f000full;
    x = (x | (x << 6)) & 0x0303030303030303ull;
    x = (x | (x << 3)) & 0x1111111111111111ull;
    return x;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    return v;
}

template <bool P, int K, class Y = Ycc, bool WAVE = false>
__device__ __forceinline__ void evaluate(const uint32_t lo[K], const uint32_t hi[K], const uint32_t pb0[K],
                                         const uint32_t pb1[K], const bool want[K], const Prob pr[K], uint32_t m0,
                                         const Y &px, const Y &tx, const EncCfg &cf, Res r[K])
{
    uint32_t a[K], b[K];
#pragma unroll
    for (int s = 0; s < K; ++s) {
        const uint32_t p1 = pr[s].mode1 ? pb0[s] : pb1[s];
        uint32_t qlo = 0, qhi = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            qlo |= ((ch(lo[s], k) << 1) | pb0[s]) << (8 * k);
            qhi |= ((ch(hi[s], k) << 1) | p1) << (8 * k);
        }
        a[s] = expand(qlo, pr[s].cbits + 1);
        b[s] = expand(qhi, pr[s].cbits + 1);
    }
    const uint32_t N = pr[0].nsel;
    const bool alpha = K == 1 && pr[0].alpha;   // only mode 6 problems carry alpha
    const uint32_t mask = K == 1 ? pr[0].mask : 0xffffu;
    uint32_t tot[K];
#pragma unroll
    for (int s = 0; s < K; ++s) tot[s] = 0;
    uint64_t ts = 0;
    const bool any_alpha = __any(alpha);
    const int w3 = alpha ? (int)cf.w[3] : 0;
    if (!P) {
        int dr[K], dg[K], db[K], da[K];
        float f[K];
#pragma unroll
        for (int s = 0; s < K; ++s) {
            dr[s] = (int)ch(b[s], 0) - (int)ch(a[s], 0);
            dg[s] = (int)ch(b[s], 1) - (int)ch(a[s], 1);
            db[s] = (int)ch(b[s], 2) - (int)ch(a[s], 2);
            da[s] = alpha ? (int)ch(b[s], 3) - (int)ch(a[s], 3) : 0;
            f[s] = N / (float)(dr[s] * dr[s] + dg[s] * dg[s] + db[s] * db[s] + da[s] * da[s] + .00000125f);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const bool f0 = first_subset<K>(m0, i);
            const uint32_t A = f0 ? a[0] : a[K - 1], B = f0 ? b[0] : b[K - 1];
            const int Dr = f0 ? dr[0] : dr[K - 1], Dg = f0 ? dg[0] : dg[K - 1], Db = f0 ? db[0] : db[K - 1];
            const float F = f0 ? f[0] : f[K - 1];
            const uint32_t c = tex(px, i);
            const int cr = ch(c, 0), cg = ch(c, 1), cb = ch(c, 2), ca = ch(c, 3);
            int dot = (cr - (int)ch(A, 0)) * Dr + (cg - (int)ch(A, 1)) * Dg + (cb - (int)ch(A, 2)) * Db;
            if (alpha) dot += (ca - (int)ch(A, 3)) * da[0];
            int sl = (int)((float)dot * F + .5f);
            sl = clampi_r(sl, 1, (int)N - 1);
            const uint32_t w0 = bc7w(sl - 1, N), w1 = bc7w(sl, N);
            int ea0 = 0, ea1 = 0;
            if (any_alpha) {   // wave-uniform: skipped by waves of opaque blocks
                const int d0 = lerp_ch(A, B, 3, w0) - ca, d1 = lerp_ch(A, B, 3, w1) - ca;
                ea0 = mad24(mul24(w3, d0), d0, 0);
                ea1 = mad24(mul24(w3, d1), d1, 0);
            }
            const uint32_t e0 =
                wsq(lerp_ch(A, B, 0, w0) - cr, lerp_ch(A, B, 1, w0) - cg, lerp_ch(A, B, 2, w0) - cb, cf, ea0);
            const uint32_t e1 =
                wsq(lerp_ch(A, B, 0, w1) - cr, lerp_ch(A, B, 1, w1) - cg, lerp_ch(A, B, 2, w1) - cb, cf, ea1);
            // both reference branches move down exactly when err0 < err1 (:479, :508)
            const bool down = e0 < e1;
            const uint32_t e = down ? e0 : e1;
            const bool in = (mask >> i) & 1u;
            tot[0] += (in && f0) ? e : 0u;
            if (K == 2) tot[K - 1] += f0 ? 0u : e;
            ts |= (uint64_t)(in ? (uint32_t)(sl - down) : 0u) << (4 * i);
        }
    } else if constexpr (WAVE) {
        // one block per wave (every lane holds it): lane L scores texel L & 15
        // against ramp points L >> 4, + 4, ... and the four lanes of a texel take
        // the minimum of (error << 4 | selector) -- the same minimum as the
        // sequential scan below (min is order-free; errors are < 2^28); the
        // subset totals are integer sums, the selectors gathered by ballots.
        const int L = (int)(threadIdx.x & 63u);
        const int i = L & 15;
        const bool f0 = first_subset<K>(m0, i);
        const uint32_t A = f0 ? a[0] : a[K - 1], B = f0 ? b[0] : b[K - 1];
        const uint32_t c = tex(px, i);
        const int tl = tx.l(i), tcr = tx.cr(i), tcb = tx.cb(i);
        uint32_t key = kNone;
        for (uint32_t j = (uint32_t)(L >> 4); j < N; j += 4) {
            const uint32_t w = bc7w(j, N);
            int l1, cr1, cb1;
            ycc_ramp(lerp_ch(A, B, 0, w), lerp_ch(A, B, 1, w), lerp_ch(A, B, 2, w), l1, cr1, cb1);
            int ea = 0;
            if (any_alpha) {   // wave-uniform; K == 1
                const int d = lerp_ch(A, B, 3, w) - (int)ch(c, 3);
                ea = mad24(mul24(w3, d), d, 0);
            }
            key = min(key, (ycc_err(l1, cr1, cb1, tl, tcr, tcb, cf, ea) << 4) | j);
        }
        key = min(key, (uint32_t)__shfl_xor((int)key, 16));
        key = min(key, (uint32_t)__shfl_xor((int)key, 32));
        const bool in = L < 16 && ((mask >> i) & 1u);
        tot[0] = wave_sum_u32((in && f0) ? key >> 4 : 0u);
        if (K == 2) tot[K - 1] = wave_sum_u32((L < 16 && !f0) ? key >> 4 : 0u);
        const uint32_t sl = in ? key & 15u : 0u;
#pragma unroll
        for (int bit = 0; bit < 4; ++bit) ts |= spread4((uint32_t)__ballot((sl >> bit) & 1u)) << bit;
    } else {
        // ramp point outer (a real loop), texels inner.  Each texel keeps the
        // minimum of (error << 4 | selector): the least error, first selector on
        // ties -- the reference's strict-< scan (:522-555); errors are < 2^28.
        uint32_t key[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) key[i] = kNone;
#pragma unroll 1
        for (uint32_t j = 0; j < N; ++j) {
            const uint32_t w = bc7w(j, N);
            int l1[K], cr1[K], cb1[K];
#pragma unroll
            for (int s = 0; s < K; ++s)
                ycc_ramp(lerp_ch(a[s], b[s], 0, w), lerp_ch(a[s], b[s], 1, w), lerp_ch(a[s], b[s], 2, w), l1[s],
                         cr1[s], cb1[s]);
            if (any_alpha) {   // wave-uniform; K == 1
                const int a1 = lerp_ch(a[0], b[0], 3, w);
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int d = a1 - (int)ch(tex(px, i), 3);
                    const uint32_t e = ycc_err(l1[0], cr1[0], cb1[0], tx.l(i), tx.cr(i), tx.cb(i), cf,
                                               mad24(mul24(w3, d), d, 0));
                    key[i] = min(key[i], (e << 4) | j);
                }
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const bool f0 = first_subset<K>(m0, i);
                    const uint32_t e = ycc_err(f0 ? l1[0] : l1[K - 1], f0 ? cr1[0] : cr1[K - 1],
                                               f0 ? cb1[0] : cb1[K - 1], tx.l(i), tx.cr(i), tx.cb(i), cf);
                    key[i] = min(key[i], (e << 4) | j);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const bool f0 = first_subset<K>(m0, i);
            const bool in = (mask >> i) & 1u;
            tot[0] += (in && f0) ? key[i] >> 4 : 0u;
            if (K == 2) tot[K - 1] += f0 ? 0u : key[i] >> 4;
            ts |= (uint64_t)(in ? key[i] & 15u : 0u) << (4 * i);
        }
    }
#pragma unroll
    for (int s = 0; s < K; ++s) {
        if (want[s] && tot[s] < r[s].err) {
            r[s].err = tot[s];
            r[s].lo = lo[s];
            r[s].hi = hi[s];
            r[s].pb0 = pb0[s];
            r[s].pb1 = pb1[s];
            r[s].sel = ts & nibble_mask(K == 1 ? mask : (s == 0 ? m0 : ~m0 & 0xffffu));
        }
    }
}

// find_optimal_solution :606-729, the endpoint quantisation (modes 1 and 6
// both carry p-bits) with fixDegenerateEndpoints :574-604 (mode 1)
__device__ __forceinline__ void quantize(float xl[4], float xh[4], const Prob &pr, uint32_t &bmin, uint32_t &bmax,
                                         uint32_t &bp0, uint32_t &bp1)
{
#pragma unroll
    for (int k = 0; k < 4; ++k) xl[k] = sat(xl[k]), xh[k] = sat(xh[k]);
    const int iscalep = (1 << (pr.cbits + 1)) - 1;
    const float scalep = (float)iscalep;
    const uint32_t nb = pr.cbits + 1;
    bmin = bmax = bp0 = bp1 = 0;
    if (!pr.mode1) {
        float be0 = 1e+9f, be1 = 1e+9f;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            uint32_t qa = 0, qb = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                qa |= (uint32_t)clampi_r(((int)((xl[k] * scalep - p) / 2.0f + .5f)) * 2 + p, p, iscalep - 1 + p)
                      << (8 * k);
                qb |= (uint32_t)clampi_r(((int)((xh[k] * scalep - p) / 2.0f + .5f)) * 2 + p, p, iscalep - 1 + p)
                      << (8 * k);
            }
            const uint32_t sa = expand(qa, nb), sb = expand(qb, nb);
            float e0 = 0, e1 = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (k == 3 && !pr.alpha) break;
                const float t0 = (int)ch(sa, k) - xl[k] * 255.0f, t1 = (int)ch(sb, k) - xh[k] * 255.0f;
                e0 += t0 * t0;
                e1 += t1 * t1;
            }
            if (e0 < be0) be0 = e0, bp0 = (uint32_t)p, bmin = (qa >> 1) & 0x7f7f7f7fu;
            if (e1 < be1) be1 = e1, bp1 = (uint32_t)p, bmax = (qb >> 1) & 0x7f7f7f7fu;
        }
    } else {
        float be = 1e+9f;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            uint32_t qa = 0, qb = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                qa |= (uint32_t)clampi_r(((int)((xl[k] * scalep - p) / 2.0f + .5f)) * 2 + p, p, iscalep - 1 + p)
                      << (8 * k);
                qb |= (uint32_t)clampi_r(((int)((xh[k] * scalep - p) / 2.0f + .5f)) * 2 + p, p, iscalep - 1 + p)
                      << (8 * k);
            }
            const uint32_t sa = expand(qa, nb), sb = expand(qb, nb);
            float e = 0;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const float t0 = ((int)ch(sa, k) / 255.0f) - xl[k], t1 = ((int)ch(sb, k) / 255.0f) - xh[k];
                e += t0 * t0 + t1 * t1;
            }
            if (e < be) be = e, bp0 = bp1 = (uint32_t)p, bmin = (qa >> 1) & 0x7f7f7f7fu, bmax = (qb >> 1) & 0x7f7f7f7fu;
        }
        const uint32_t isc = (uint32_t)(iscalep >> 1);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            uint32_t mn = ch(bmin, k), mx = ch(bmax, k);
            if (mn != mx || !(fabsf(xl[k] - xh[k]) > 0.0f)) continue;
            if (mn > (isc >> 1)) {
                if (mn > 0)
                    mn--;
                else if (mx < isc)
                    mx++;
            } else {
                if (mx < isc)
                    mx++;
                else if (mn > 0)
                    mn--;
            }
            bmin = (bmin & ~(0xffu << (8 * k))) | (mn << (8 * k));
            bmax = (bmax & ~(0xffu << (8 * k))) | (mx << (8 * k));
        }
    }
}

// find_optimal_solution for the K problems: quantise each active one's
// endpoints, evaluate those that differ from its best (:710, :724)
template <bool P, int K, class Y = Ycc, bool WAVE = false>
__device__ __forceinline__ void fit(float xl[K][4], float xh[K][4], const bool active[K], const Prob pr[K],
                                    uint32_t m0, const Y &px, const Y &tx, const EncCfg &cf, Res r[K])
{
    uint32_t lo[K], hi[K], p0[K], p1[K];
    bool want[K], any = false;
#pragma unroll
    for (int s = 0; s < K; ++s) {
        quantize(xl[s], xh[s], pr[s], lo[s], hi[s], p0[s], p1[s]);
        want[s] = active[s] && (r[s].err == kNone || lo[s] != r[s].lo || hi[s] != r[s].hi || p0[s] != r[s].pb0 ||
                                p1[s] != r[s].pb1);
        any = any || want[s];
    }
    if (any) evaluate<P, K, Y, WAVE>(lo, hi, p0, p1, want, pr, m0, px, tx, cf, r);
}

// compute_least_squares_endpoints_rgb / _rgba :197-280 for the K problems in
// one texel pass (each texel adds to its own subset's sums, in texel order),
// then the 1/255 scale
template <int K, class Y>
__device__ __forceinline__ void lsq(const Prob pr[K], uint32_t m0, uint64_t sel, const Y &px,
                                    const EncLds &L, float xl[K][4], float xh[K][4])
{
    const float *wx = L.wx + (pr[0].nsel == 16 ? 32 : 0);
    const bool need_a = K == 1 && __any(pr[0].alpha);   // wave-uniform; mode-1 problems are opaque
    float z00[K], z10[K], z11[K], q00[K][4], t[K][4];
#pragma unroll
    for (int s = 0; s < K; ++s) {
        z00[s] = z10[s] = z11[s] = 0.0f;
#pragma unroll
        for (int k = 0; k < 4; ++k) q00[s][k] = t[s][k] = 0.0f;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const bool f0 = first_subset<K>(m0, i);
        const bool in = K == 2 || ((pr[0].mask >> i) & 1u);
        const float *w4 = wx + 4 * sel_at(sel, i);
        const float w = w4[3];
        uint32_t c[4];
        px.chans(i, need_a, c);
#pragma unroll
        for (int s = 0; s < K; ++s) {
            const bool add = in && (s == 0 ? f0 : !f0);
            z00[s] = add ? z00[s] + w4[0] : z00[s];
            z10[s] = add ? z10[s] + w4[1] : z10[s];
            z11[s] = add ? z11[s] + w4[2] : z11[s];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (k == 3 && !need_a) break;   // (alpha sums are only read by alpha problems)
                const float v = (float)c[k];
                q00[s][k] = add ? q00[s][k] + w * v : q00[s][k];
                t[s][k] = add ? t[s][k] + v : t[s][k];
            }
        }
    }
#pragma unroll
    for (int s = 0; s < K; ++s) {
        const float z01 = z10[s];
        float det = z00[s] * z11[s] - z01 * z10[s];
        if (det != 0.0f) det = 1.0f / det;
        const float i00 = z11[s] * det, i01 = -z01 * det, i10 = -z10[s] * det, i11 = z00[s] * det;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float q10 = t[s][k] - q00[s][k];
            float l = i00 * q00[s][k] + i01 * q10, h = i10 * q00[s][k] + i11 * q10;
            if (k == 3 && !pr[s].alpha) l = h = 255.0f;
            xl[s][k] = l * (1.0f / 255.0f);
            xh[s][k] = h * (1.0f / 255.0f);
        }
    }
}

// pack_mode1_to_one_color :357-403
template <bool P, class Y = Ycc>
__device__ __forceinline__ void one_colour(uint32_t cr, uint32_t cg, uint32_t cb, const Prob &pr, const Y &px, const Y &tx,
                           const EncCfg &cf, const EncLds &L, Res &r)
{
    uint32_t best = kNone, bp = 0;
#pragma unroll
    for (uint32_t p = 0; p < 2; ++p) {
        const uint32_t e = (L.one[cr * 2 + p] & 0xffffu) + (L.one[cg * 2 + p] & 0xffffu) + (L.one[cb * 2 + p] & 0xffffu);
        if (e < best) best = e, bp = p;
    }
    const uint32_t er = L.one[cr * 2 + bp], eg = L.one[cg * 2 + bp], eb = L.one[cb * 2 + bp];
    r.lo = ((er >> 16) & 0xffu) | (((eg >> 16) & 0xffu) << 8) | (((eb >> 16) & 0xffu) << 16);
    r.hi = (er >> 24) | ((eg >> 24) << 8) | ((eb >> 24) << 16);
    r.pb0 = bp;
    r.pb1 = 0;
    int q[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        uint32_t lo = ((ch(r.lo, k) << 1) | bp) << 1;
        lo |= lo >> 7;
        uint32_t hi = ((ch(r.hi, k) << 1) | bp) << 1;
        hi |= hi >> 7;
        q[k] = (int)((lo * (64u - 18u) + hi * 18u + 32u) >> 6);
    }
    int ql, qcr, qcb;
    ycc_ramp(q[0], q[1], q[2], ql, qcr, qcb);
    uint32_t tot = 0;
    uint64_t ts = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t c = tex(px, i);
        const uint32_t e = P ? ycc_err(ql, qcr, qcb, tx.l(i), tx.cr(i), tx.cb(i), cf)
                             : wsq(q[0] - (int)ch(c, 0), q[1] - (int)ch(c, 1), q[2] - (int)ch(c, 2), cf);
        const bool in = (pr.mask >> i) & 1u;
        tot += in ? e : 0u;
        ts |= (uint64_t)(in ? 2u : 0u) << (4 * i);
    }
    r.sel = ts;
    r.err = tot;
}

// the subset's channel sums in texel order (exact: integers below 2^24)
template <class Y>
__device__ __forceinline__ void subset_sums(const Prob &pr, const Y &px, float m[4])
{
#pragma unroll
    for (int k = 0; k < 4; ++k) m[k] = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const bool in = (pr.mask >> i) & 1u;
#pragma unroll
        for (int k = 0; k < 4; ++k) m[k] = in ? m[k] + (float)ch(tex(px, i), k) : m[k];
    }
}

// the subset mean as color_cell_compression scales it (:766-771)
template <class Y>
__device__ __forceinline__ void subset_mean(const Prob &pr, const Y &px, float mn[4])
{
    float m[4];
    subset_sums(pr, px, m);
    const float inv_n255 = 1.0f / (float)(pr.n * 255.0f);
#pragma unroll
    for (int k = 0; k < 4; ++k) mn[k] = sat(m[k] * inv_n255);
}

// color_cell_compression :756-874: the subset's mean and principal axis, and the
// PCA endpoints the first fit starts from
template <bool P, class Y>
__device__ __forceinline__ void pca_endpoints(const Prob &pr, const Y &px, float cmin[4], float cmax[4])
{
    // mean and principal axis (:756-841)
    float m[4], mn[4];
    subset_sums(pr, px, m);
    float ms[4], ax[4] = {0.f, 0.f, 0.f, 0.f};
    const float inv_n = 1.0f / (float)pr.n, inv_n255 = 1.0f / (float)(pr.n * 255.0f);
#pragma unroll
    for (int k = 0; k < 4; ++k) ms[k] = m[k] * inv_n, mn[k] = sat(m[k] * inv_n255);
    if (pr.alpha) {   // incremental PCA (:773-790); alpha problems are whole blocks (mode 6)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            float c[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) c[k] = (float)ch(tex(px, i), k) - ms[k];
            float n[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) n[k] = i ? ax[k] : c[k];
            float s = n[0] * n[0] + n[1] * n[1] + n[2] * n[2] + n[3] * n[3];
            if (s != 0.0f) {
                s = 1.0f / sqrtf(s);
#pragma unroll
                for (int k = 0; k < 4; ++k) n[k] *= s;
            }
            float add[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float a0 = c[0] * c[q], a1 = c[1] * c[q], a2 = c[2] * c[q], a3 = c[3] * c[q];
                add[q] = a0 * n[0] + a1 * n[1] + a2 * n[2] + a3 * n[3];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) ax[q] += add[q];
        }
        float s = ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2] + ax[3] * ax[3];
        if (s != 0.0f) {
            s = 1.0f / sqrtf(s);
#pragma unroll
            for (int k = 0; k < 4; ++k) ax[k] *= s;
        }
    } else {   // covariance and three power steps (:795-831)
        float cv[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const bool in = (pr.mask >> i) & 1u;
            const float r0 = (int)ch(tex(px, i), 0) - ms[0], g0 = (int)ch(tex(px, i), 1) - ms[1], b0 = (int)ch(tex(px, i), 2) - ms[2];
            const float t[6] = {r0 * r0, r0 * g0, r0 * b0, g0 * g0, g0 * b0, b0 * b0};
#pragma unroll
            for (int k = 0; k < 6; ++k) cv[k] = in ? cv[k] + t[k] : cv[k];
        }
        float vr = .9f, vg = 1.0f, vb = .7f;
#pragma unroll
        for (int it = 0; it < 3; ++it) {
            float x = vr * cv[0] + vg * cv[1] + vb * cv[2];
            float y = vr * cv[1] + vg * cv[3] + vb * cv[4];
            float z = vr * cv[2] + vg * cv[4] + vb * cv[5];
            const float ax0 = fabsf(x), ay0 = fabsf(y), az0 = fabsf(z);
            const float mxy = ax0 > ay0 ? ax0 : ay0;
            float mm = mxy > az0 ? mxy : az0;
            if (mm > 1e-10f) {
                mm = 1.0f / mm;
                x *= mm, y *= mm, z *= mm;
            }
            vr = x, vg = y, vb = z;
        }
        float len = vr * vr + vg * vg + vb * vb;
        if (!(len < 1e-10f)) {
            len = 1.0f / sqrtf(len);
            ax[0] = vr * len, ax[1] = vg * len, ax[2] = vb * len;
        }
    }
    if (ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2] + ax[3] * ax[3] < .5f) {
        if (P)
            ax[0] = .213f, ax[1] = .715f, ax[2] = .072f, ax[3] = pr.alpha ? .715f : 0.f;
        else
            ax[0] = 1.0f, ax[1] = 1.0f, ax[2] = 1.0f, ax[3] = pr.alpha ? 1.0f : 0.f;
        float s = ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2] + ax[3] * ax[3];
        if (s != 0.0f) {
            s = 1.0f / sqrtf(s);
#pragma unroll
            for (int k = 0; k < 4; ++k) ax[k] *= s;
        }
    }
    float lo = 1e+9f, hi = -1e+9f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const bool in = (pr.mask >> i) & 1u;
        float q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = (float)ch(tex(px, i), k) - ms[k];
        const float d = q[0] * ax[0] + q[1] * ax[1] + q[2] * ax[2] + q[3] * ax[3];
        lo = (in && !(lo < d)) ? d : lo;
        hi = (in && !(hi > d)) ? d : hi;
    }
    lo *= (1.0f / 255.0f);
    hi *= (1.0f / 255.0f);
#pragma unroll
    for (int k = 0; k < 4; ++k) cmin[k] = sat(mn[k] + ax[k] * lo), cmax[k] = sat(mn[k] + ax[k] * hi);
    if (cmin[0] * 1.0f + cmin[1] * 1.0f + cmin[2] * 1.0f + cmin[3] * 1.0f >
        cmax[0] * 1.0f + cmax[1] * 1.0f + cmax[2] * 1.0f + cmax[3] * 1.0f) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float t = cmin[k];
            cmin[k] = cmax[k];
            cmax[k] = t;
        }
    }

}

// color_cell_compression :731-1024 for K problems in lockstep
template <bool P, int K, class Y = Ycc, bool WAVE = false>
__device__ __forceinline__ void cells(const Prob pr[K], uint32_t m0, const Y &px, const Y &tx,
                                      const EncCfg &cf, const EncLds &L, Res r[K])
{
    bool fin[K];   // the subset was packed as one colour (:738-754): no trials
#pragma unroll
    for (int s = 0; s < K; ++s) {
        r[s].err = kNone;
        r[s].lo = r[s].hi = r[s].pb0 = r[s].pb1 = 0;
        r[s].sel = 0;
        fin[s] = false;
        if (pr[s].mode1) {
            uint32_t first = 0;
            bool same = true;
#pragma unroll
            for (int i = 15; i >= 0; --i) first = ((pr[s].mask >> i) & 1u) ? tex(px, i) & 0xffffffu : first;
#pragma unroll
            for (int i = 0; i < 16; ++i)
                same = same && (!((pr[s].mask >> i) & 1u) || (tex(px, i) & 0xffffffu) == first);
            if (same) {
                one_colour<P>(ch(first, 0), ch(first, 1), ch(first, 2), pr[s], px, tx, cf, L, r[s]);
                fin[s] = true;
            }
        }
    }

    // Trials, each a fit that keeps the best (:874-1006): t = 0 the PCA endpoints;
    // then the least-squares refit of the current selectors; uber >= 1: refits of
    // the snapshot with its minimum selectors raised, its maximum lowered, both;
    // uber >= 2 and error above (n*56)>>4: refits of rescaled snapshots over
    // ly in [-Q, 1] x hy in [max-1, max+Q] without (0, max).
    const int nls = cf.lsq ? 1 : 0;
    const int nub = cf.uber > 0 ? 3 : 0;
    const int Q = cf.uber >= 4 ? (int)cf.uber - 2 : 1;
    const int ngrid = cf.uber >= 2 ? (Q + 2) * (Q + 2) - 1 : 0;
    const int ntr = 1 + nls + nub + ngrid;
    const int maxs = (int)pr[0].nsel - 1;
    bool zero[K], grid[K];
    uint32_t smin[K], smax[K];
    uint64_t base = 0;
#pragma unroll
    for (int s = 0; s < K; ++s) zero[s] = grid[s] = false, smin[s] = 16, smax[s] = 0;
    for (int t = 0; t < ntr; ++t) {
        if (t == 1 + nls) {   // the uber snapshot: each subset's selectors sit in its own nibbles
            base = 0;
#pragma unroll
            for (int s = 0; s < K; ++s) base |= r[s].sel;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const bool f0 = first_subset<K>(m0, i);
                const uint32_t v = sel_at(base, i);
#pragma unroll
                for (int s = 0; s < K; ++s) {
                    const bool mine = (s == 0 ? f0 : !f0) && (K == 2 || ((pr[0].mask >> i) & 1u));
                    smin[s] = mine && v < smin[s] ? v : smin[s];
                    smax[s] = mine && v > smax[s] ? v : smax[s];
                }
            }
        }
        bool active[K], any = false;
#pragma unroll
        for (int s = 0; s < K; ++s) {
            if (t == 1 + nls + nub) grid[s] = r[s].err > ((pr[s].n * 56u) >> 4);
            active[s] = !fin[s] && !zero[s] && (t < 1 + nls + nub || grid[s]);
            any = any || active[s];
        }
        if (!any) break;   // color_cell_compression returned (0) or finished its trials
        float xl[K][4], xh[K][4];
        if (t == 0) {
            // the PCA endpoints, computed here so that nothing of them stays live
            // through the trials (register budget)
#pragma unroll
            for (int s = 0; s < K; ++s) {
#pragma unroll
                for (int k = 0; k < 4; ++k) xl[s][k] = xh[s][k] = 0.f;
                if (active[s]) pca_endpoints<P, Y>(pr[s], px, xl[s], xh[s]);
            }
        } else {
            uint64_t ts = 0;
            if (t <= nls) {
#pragma unroll
                for (int s = 0; s < K; ++s) ts |= r[s].sel;
            } else if (t < 1 + nls + nub) {
                // texels outside the problems get some selector in 0..15 that lsq ignores
                const int u = t - 1 - nls;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const bool f0 = first_subset<K>(m0, i);
                    const uint32_t lo_s = f0 ? smin[0] : smin[K - 1], hi_s = f0 ? smax[0] : smax[K - 1];
                    uint32_t v = sel_at(base, i);
                    if (u != 1 && v == lo_s && v < pr[0].nsel - 1)
                        v++;
                    else if (u != 0 && v == hi_s && v > 0)
                        v--;
                    ts |= (uint64_t)v << (4 * i);
                }
            } else {
                int g = t - (1 + nls + nub);
                if (g >= Q * (Q + 2) + 1) ++g;   // skip (ly, hy) = (0, max)
                const int ly = -Q + g / (Q + 2), hy = maxs - 1 + g % (Q + 2);
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const float v = floorf((float)maxs * ((float)sel_at(base, i) - (float)ly) / ((float)hy - (float)ly) +
                                           .5f);
                    ts |= (uint64_t)(uint32_t)clampf_r(v, 0, (float)maxs) << (4 * i);
                }
            }
            lsq<K, Y>(pr, m0, ts, px, L, xl, xh);
        }
        fit<P, K, Y, WAVE>(xl, xh, active, pr, m0, px, tx, cf, r);
#pragma unroll
        for (int s = 0; s < K; ++s) zero[s] = zero[s] || (active[s] && r[s].err == 0);
    }
#pragma unroll
    for (int s = 0; s < K; ++s) {
        if (pr[s].mode1 && !fin[s] && !zero[s]) {   // the subset mean as one colour (:1009-1021)
            Res avg = r[s];
            float mn[4];
            subset_mean(pr[s], px, mn);   // recomputed: the same sums as pca_endpoints'
            one_colour<P>((uint32_t)(int)(.5f + mn[0] * 255.0f), (uint32_t)(int)(.5f + mn[1] * 255.0f),
                          (uint32_t)(int)(.5f + mn[2] * 255.0f), pr[s], px, tx, cf, L, avg);
            if (avg.err < r[s].err) r[s] = avg;
        }
    }
}

// color_cell_compression_est :1026-1162 for both subsets of a two-subset shape
// in one pass (m0 = the texels of subset 0): bounding-box endpoints, 8 ramp
// points, selectors by dot-product thresholds.  The reference stops a sum once
// it exceeds the best so far; its caller only compares with '<', so full sums
// are equivalent.
struct EstSubset {
    int lo[3], hi[3], a[3], th[7];
};

__device__ __forceinline__ void est_setup(EstSubset &e)
{
#pragma unroll
    for (int k = 0; k < 3; ++k) e.a[k] = e.hi[k] - e.lo[k];
    int prev = e.lo[0] * e.a[0] + e.lo[1] * e.a[1] + e.lo[2] * e.a[2];
#pragma unroll
    for (int s = 1; s < 8; ++s) {
        const int w = (int)bc7w((uint32_t)s, 8);
        int d = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) d += ((e.lo[k] * (64 - w) + e.hi[k] * w + 32) >> 6) * e.a[k];
        e.th[s - 1] = (prev + d + 1) >> 1;
        prev = d;
    }
}

//
// `best` is the least total so far: once every lane of the wave has a partial
// sum at or above its own best, the rest cannot make the shape win (the terms
// are non-negative and the caller keeps a total only if it is strictly less),
// so the sum stops -- the reference's own early exit (:1156-1157), taken per
// wave after every two texels.
// The block's texel words in registers, for the partition estimate's phase
// (its shapes re-read every texel; nothing of the trials is live then).
struct RegTex {
    uint32_t w[16];
    template <class Y>
    __device__ __forceinline__ void load(const Y &y)
    {
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = y.word(i);
    }
    __device__ __forceinline__ uint32_t word(int i) const
    {
        uint32_t v = w[i];
        asm volatile("" : "+v"(v));   // new at every use: keeps the channel conversions out of the shape loop
        return v;
    }
};

template <bool P, class Y = Ycc>
__device__ __forceinline__ uint32_t estimate2(uint32_t m0, const RegTex &px, const Y &tx, const EncCfg &cf,
                                              uint32_t best)
{
    EstSubset s0, s1;
#pragma unroll
    for (int k = 0; k < 3; ++k) s0.lo[k] = s1.lo[k] = 255, s0.hi[k] = s1.hi[k] = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const bool in0 = (m0 >> i) & 1u;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int v = ch(tex(px, i), k);
            s0.lo[k] = in0 && v < s0.lo[k] ? v : s0.lo[k];
            s0.hi[k] = in0 && v > s0.hi[k] ? v : s0.hi[k];
            s1.lo[k] = !in0 && v < s1.lo[k] ? v : s1.lo[k];
            s1.hi[k] = !in0 && v > s1.hi[k] ? v : s1.hi[k];
        }
    }
    est_setup(s0);
    est_setup(s1);
    uint32_t tot = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if ((i & 1) == 0 && i > 0 && __all(tot >= best)) break;
        const bool in0 = (m0 >> i) & 1u;
        int lo[3], hi[3], th[7];
        int d = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            lo[k] = in0 ? s0.lo[k] : s1.lo[k];
            hi[k] = in0 ? s0.hi[k] : s1.hi[k];
            d += (in0 ? s0.a[k] : s1.a[k]) * (int)ch(tex(px, i), k);
        }
        int s = 0;   // the ramp's dots rise with s: the first threshold from the top is a count
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            th[k] = in0 ? s0.th[k] : s1.th[k];
            s += d >= th[k];
        }
        const int w = (int)bc7w((uint32_t)s, 8);
        int c[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) c[k] = (lo[k] * (64 - w) + hi[k] * w + 32) >> 6;
        if (P) {
            int l1, cr1, cb1;
            ycc_ramp(c[0], c[1], c[2], l1, cr1, cb1);
            tot += ycc_err(l1, cr1, cb1, tx.l(i), tx.cr(i), tx.cb(i), cf);
        } else {
            tot += wsq(c[0] - (int)ch(tex(px, i), 0), c[1] - (int)ch(tex(px, i), 1), c[2] - (int)ch(tex(px, i), 2), cf);
        }
    }
    return tot;
}

__device__ __forceinline__ uint32_t shape_mask(uint32_t shape, uint32_t subset)
{
    uint32_t m = 0;
#pragma unroll
    for (int t = 0; t < 16; ++t) m |= (((shape >> (2 * t)) & 3u) == subset ? 1u : 0u) << t;
    return m;
}

// estimate_partition :1207-1281
template <bool P, class Y = Ycc>
__device__ __forceinline__ uint32_t pick_partition(const Y &tx, const EncCfg &cf)
{
    const uint32_t total = cf.max_parts < 64 ? cf.max_parts : 64;
    if (total <= 1) return 0;
    RegTex px;
    px.load(tx);
    uint32_t best = kNone, best_part = 0, key = 0;
    bool stop = false;
    for (uint32_t it = 0; it < total; ++it) {
        if (stop || best == 0) break;
        const uint32_t part = kEncPartOrder[it];
        if (cf.filterbank && it >= 14 && it <= 34 && !(kEncPredictors[part] & (1u << (key + 1)))) {
            if (it == 34) stop = true;
            continue;
        }
        const uint32_t m0 = shape_mask(kBc7Shape2[part], 0);
        const uint32_t e = estimate2<P>(m0, px, tx, cf, best);
        if (e < best) best = e, best_part = part;
        if (part == 34 && best_part != 34) stop = true;
        if (it == 13) key = best_part;
    }
    return best_part;
}

// pick_partition with the shapes' estimates on the lanes of a wave (one block per
// wave, every lane holding it): lane it sums shape kEncPartOrder[it] in full, then
// the reference's sequential choice (filter bank, stop rules, '<' keeps the
// first) runs over those totals -- full sums are equivalent (see estimate2).
template <bool P, class Y = Ycc>
__device__ __forceinline__ uint32_t pick_partition_wave(const Y &tx, const EncCfg &cf)
{
    const uint32_t total = cf.max_parts < 64 ? cf.max_parts : 64;
    if (total <= 1) return 0;
    RegTex px;
    px.load(tx);
    const uint32_t ln = threadIdx.x & 63u;
    uint32_t el = kNone;
    if (ln < total) el = estimate2<P>(shape_mask(kBc7Shape2[kEncPartOrder[ln]], 0), px, tx, cf, kNone);
    uint32_t best = kNone, best_part = 0, key = 0;
    bool stop = false;
    for (uint32_t it = 0; it < total; ++it) {
        if (stop || best == 0) break;
        const uint32_t part = kEncPartOrder[it];
        if (cf.filterbank && it >= 14 && it <= 34 && !(kEncPredictors[part] & (1u << (key + 1)))) {
            if (it == 34) stop = true;
            continue;
        }
        const uint32_t e = (uint32_t)__builtin_amdgcn_readlane((int)el, (int)it);   // it: wave-uniform
        if (e < best) best = e, best_part = part;
        if (part == 34 && best_part != 34) stop = true;
        if (it == 13) key = best_part;
    }
    return best_part;
}

// 128-bit little-endian bit writer (set_block_bits :1283-1295)
struct Bits {
    uint64_t w0 = 0, w1 = 0;
    uint32_t pos = 0;
    __device__ void put(uint32_t v, uint32_t n)
    {
        const uint64_t x = (uint64_t)v;
        if (pos < 64) {
            w0 |= x << pos;
            if (pos + n > 64) w1 |= x >> (64 - pos);
        } else {
            w1 |= x << (pos - 64);
        }
        pos += n;
    }
};

// encode_bc7_block :1307-1388 for mode 6 (one subset) or mode 1 (partition `part`)
__device__ __forceinline__ uint4 pack_block(bool mode1, uint32_t part, uint64_t sel, const uint32_t lo[2], const uint32_t hi[2],
                            uint32_t pb[2][2])
{
    const uint32_t shape = mode1 ? kBc7Shape2[part] : 0u;
    const uint32_t ib = mode1 ? 3 : 4, nsub = mode1 ? 2 : 1;
    const uint32_t anc1 = mode1 ? kBc7Anchor2[part] : 0xffu;
    uint32_t l[2] = {lo[0], lo[1]}, h[2] = {hi[0], hi[1]};
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) {
        if (k >= nsub) break;
        const uint32_t a = k ? anc1 : 0;
        if (!((uint32_t)(sel >> (4 * a)) & (1u << (ib - 1)))) continue;
#pragma unroll
        for (int t = 0; t < 16; ++t)
            if (((shape >> (2 * t)) & 3u) == k) sel ^= (uint64_t)((1u << ib) - 1) << (4 * t);
        const uint32_t tl = l[k];
        l[k] = h[k];
        h[k] = tl;
        if (!mode1) {
            const uint32_t tp = pb[k][0];
            pb[k][0] = pb[k][1];
            pb[k][1] = tp;
        }
    }
    Bits b;
    if (mode1) {
        b.put(2u, 2);
        b.put(part, 6);
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
            for (int k = 0; k < 2; ++k) b.put(ch(l[k], c), 6), b.put(ch(h[k], c), 6);
        b.put(pb[0][0], 1);
        b.put(pb[1][0], 1);
#pragma unroll
        for (int t = 0; t < 16; ++t) b.put(sel_at(sel, t), (t == 0 || (uint32_t)t == anc1) ? 2 : 3);
    } else {
        b.put(64u, 7);
#pragma unroll
        for (int c = 0; c < 4; ++c) b.put(ch(l[0], c), 7), b.put(ch(h[0], c), 7);
        b.put(pb[0][0], 1);
        b.put(pb[0][1], 1);
#pragma unroll
        for (int t = 0; t < 16; ++t) b.put(sel_at(sel, t), t == 0 ? 3 : 4);
    }
    return make_uint4((uint32_t)b.w0, (uint32_t)(b.w0 >> 32), (uint32_t)b.w1, (uint32_t)(b.w1 >> 32));
}

// bc7enc16_compress_block :1517-1547 with handle_alpha_block / handle_opaque_block
// :1390-1515 (m_endpoints_share_pbit, uninitialised for alpha blocks in the
// reference, is false: mode 6 has a p-bit per endpoint)
template <bool P, bool WAVE = false, class Y = Ycc>
__device__ __forceinline__ void encode_block(const uint32_t px[16], const EncCfg &cf, const EncLds &L, Y tx,
                                             uint4 *out, bool writer)
{
    // the texels go to LDS (YccT / TexT); the register copy dies here
#pragma unroll
    for (int i = 0; i < 16; ++i) tx.put(i, px[i]);
    bool alpha = false;
#pragma unroll
    for (int i = 0; i < 16; ++i) alpha = alpha || (px[i] >> 24) < 255u;
    uint32_t err6;
    {   // mode 6 on the whole block
        Prob p6[1];
        Res r6[1];
        p6[0].mask = 0xffffu, p6[0].n = 16, p6[0].nsel = 16, p6[0].cbits = 7, p6[0].mode1 = false, p6[0].alpha = alpha;
        cells<P, 1, Y, WAVE>(p6, 0xffffu, tx, tx, cf, L, r6);
        // the mode-6 block goes out now and is overwritten if mode 1 wins: only
        // its error stays live through the mode-1 search (register budget)
        const uint32_t lo[2] = {r6[0].lo, 0}, hi[2] = {r6[0].hi, 0};
        uint32_t pb[2][2] = {{r6[0].pb0, r6[0].pb1}, {0, 0}};
        const uint4 b6 = pack_block(false, 0, r6[0].sel, lo, hi, pb);
        if (writer) *out = b6;
        err6 = r6[0].err;
    }
    if (!alpha && err6 > 0 && cf.max_parts > 0) {
        // mode 1 on the partition the estimator picks, both subsets at once (the
        // reference stops after the first subset if it alone loses: equivalent)
        const uint32_t part = WAVE ? pick_partition_wave<P>(tx, cf) : pick_partition<P>(tx, cf);
        const uint32_t m0 = shape_mask(kBc7Shape2[part], 0);
        Prob p1[2];
        Res r1[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            p1[k].mask = k ? (~m0 & 0xffffu) : m0;
            p1[k].n = (uint32_t)__popc(p1[k].mask), p1[k].nsel = 8, p1[k].cbits = 6, p1[k].mode1 = true;
            p1[k].alpha = false;
        }
        cells<P, 2, Y, WAVE>(p1, m0, tx, tx, cf, L, r1);
        if (r1[0].err + r1[1].err < err6) {
            // each subset's selectors sit in its own texels' nibbles
            const uint32_t lo[2] = {r1[0].lo, r1[1].lo}, hi[2] = {r1[0].hi, r1[1].hi};
            uint32_t pb[2][2] = {{r1[0].pb0, 0}, {r1[1].pb0, 0}};
            const uint4 b1 = pack_block(true, part, r1[0].sel | r1[1].sel, lo, hi, pb);
            if (writer) *out = b1;
        }
    }
}

// ---- kernels ---------------------------------------------------------------

// waves per SIMD the kernels are register-budgeted for (build-time override for
// studies).  3: with the perceptual transforms in LDS the 3-wave build spills
// only values read once per block (the PCA endpoints, the cfg); 8K G1 uber 4
// perceptual 32.8 -> 32.0 ms, uber 0 12.9 -> 12.2 ms, RGB metric 20.0 -> 18.0 ms
// and 11.2 -> 10.3 ms against the 2-wave build, same blocks
// (profiles/r04c_bc7enc_ab.txt)
#ifndef GIC_ENC_WAVES
#define GIC_ENC_WAVES 3
#endif

__device__ __forceinline__ void load_tables(EncLds &L)
{
    for (uint32_t i = threadIdx.x; i < 96; i += blockDim.x)
        L.wx[i] = __uint_as_float(i < 32 ? kEncW3x[i] : kEncW4x[i - 32]);
    for (uint32_t i = threadIdx.x; i < 512; i += blockDim.x) L.one[i] = kEncOneColour[i];
    __syncthreads();
}

// Image_CompressRichGel999BC7 :21-71 over 8-bit texels (its float round trip
// v/255.0f -> R8G8B8A8_UNORM gives back the bytes)
template <bool P>
__global__ void __launch_bounds__(256, GIC_ENC_WAVES) bc7enc_image_kernel(Geometry g, EncCfg cf, int force_alpha_one,
                                                           uint4 *__restrict__ dst)
{
    __shared__ EncLds L;
    __shared__ int ytab[TexSrc<P, kYccStride>::kRows * kYccStride];
    load_tables(L);
    const TexSrc<P, kYccStride> tx{(uint32_t)(uintptr_t)(const __attribute__((address_space(3))) int *)(ytab + threadIdx.x)};
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= g.total) return;
    uint32_t slice, by, bx;
    block_coords(g, id, slice, by, bx);
    uint32_t px[16];
    load_block_u8(g, slice, by, bx, force_alpha_one != 0, px);
    encode_block<P>(px, cf, L, tx, dst + id, true);
}

// Image_CompressRichGel999BC7enc16 :73-97: blocks of 16 packed RGBA8 words
template <bool P>
__global__ void __launch_bounds__(256, GIC_ENC_WAVES) bc7enc_blocks_kernel(const uint4 *__restrict__ blocks, uint32_t n, EncCfg cf,
                                                            uint4 *__restrict__ dst)
{
    __shared__ EncLds L;
    __shared__ int ytab[TexSrc<P, kYccStride>::kRows * kYccStride];
    load_tables(L);
    const TexSrc<P, kYccStride> tx{(uint32_t)(uintptr_t)(const __attribute__((address_space(3))) int *)(ytab + threadIdx.x)};
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= n) return;
    uint32_t px[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint4 v = blocks[(size_t)id * 4 + q];
        px[q * 4 + 0] = v.x, px[q * 4 + 1] = v.y, px[q * 4 + 2] = v.z, px[q * 4 + 3] = v.w;
    }
    encode_block<P>(px, cf, L, tx, dst + id, true);
}

// small batches (the block-level entry point): one block per 64-lane wave, the
// mode-1 partition estimates on the lanes (pick_partition_wave)
template <bool P>
__global__ void __launch_bounds__(64) bc7enc_blocks_wave_kernel(const uint4 *__restrict__ blocks, uint32_t n, EncCfg cf,
                                                                uint4 *__restrict__ dst)
{
    __shared__ EncLds L;
    __shared__ int ytab[TexSrc<P, 64>::kRows * 64];
    load_tables(L);
    const TexSrc<P, 64> tx{(uint32_t)(uintptr_t)(const __attribute__((address_space(3))) int *)(ytab + threadIdx.x)};
    const uint32_t id = blockIdx.x;
    if (id >= n) return;
    uint32_t px[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint4 v = blocks[(size_t)id * 4 + q];
        px[q * 4 + 0] = v.x, px[q * 4 + 1] = v.y, px[q * 4 + 2] = v.z, px[q * 4 + 3] = v.w;
    }
    encode_block<P, true>(px, cf, L, tx, dst + id, threadIdx.x == 0);
}

// float RGBA blocks (the gic_hip_encode_rows_src / block-ABI path): each texel
// to RGBA8 as saturate(v) * 255 + 0.5 truncated (TinyImageFormat's UNORM8 encode
// is un-vendored; this rounding is unpinned and is the identity on v / 255.0f)
template <bool P>
__global__ void __launch_bounds__(256, GIC_ENC_WAVES) bc7enc_f32_kernel(const float *__restrict__ blocks, uint32_t n, EncCfg cf,
                                                         uint4 *__restrict__ dst)
{
    __shared__ EncLds L;
    __shared__ int ytab[TexSrc<P, kYccStride>::kRows * kYccStride];
    load_tables(L);
    const TexSrc<P, kYccStride> tx{(uint32_t)(uintptr_t)(const __attribute__((address_space(3))) int *)(ytab + threadIdx.x)};
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= n) return;
    uint32_t px[16];
    const float4 *b = reinterpret_cast<const float4 *>(blocks) + (size_t)id * 16;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        const float4 v = b[t];
        const float c[4] = {v.x, v.y, v.z, v.w};
        uint32_t w = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) w |= (uint32_t)(sat(c[k]) * 255.0f + 0.5f) << (8 * k);
        px[t] = w;
    }
    encode_block<P>(px, cf, L, tx, dst + id, true);
}

EncCfg make_cfg(const gic_options &o)
{
    EncCfg c;
    c.uber = o.bc7enc_uber_level;
    c.max_parts = o.bc7enc_max_partitions;
    c.lsq = o.bc7enc_least_squares;
    c.filterbank = o.bc7enc_filterbank;
    if (o.bc7enc_perceptual) {   // bc7enc16_compress_block_params_init_perceptual_weights + :1524-1532
        const volatile float pr = (.5f / (1.0f - .2126f)) * (.5f / (1.0f - .2126f));
        const volatile float pb = (.5f / (1.0f - .0722f)) * (.5f / (1.0f - .0722f));
        c.w[0] = (uint32_t)(int)(128u * 4.0f);
        c.w[1] = (uint32_t)(int)(64u * 4.0f * pr);
        c.w[2] = (uint32_t)(int)(16u * 4.0f * pb);
        c.w[3] = 32u * 4u;
    } else {
        c.w[0] = c.w[1] = c.w[2] = c.w[3] = 1;
    }
    return c;
}

}  // namespace

hipError_t launch_bc7enc_image(const Geometry &g, const gic_options &o, void *dst, hipStream_t s)
{
    const EncCfg cf = make_cfg(o);
    const uint32_t wg = 256, grid = (g.total + wg - 1) / wg;
    const int fa = o.force_alpha_one || g.channels < 4;
    if (o.bc7enc_perceptual)
        hipLaunchKernelGGL(bc7enc_image_kernel<true>, dim3(grid), dim3(wg), 0, s, g, cf, fa, (uint4 *)dst);
    else
        hipLaunchKernelGGL(bc7enc_image_kernel<false>, dim3(grid), dim3(wg), 0, s, g, cf, fa, (uint4 *)dst);
    return hipGetLastError();
}

hipError_t launch_bc7enc_blocks_u8(const uint32_t *blocks, uint32_t n, const gic_options &o, void *dst, hipStream_t s)
{
    const EncCfg cf = make_cfg(o);
    if (n < 4096) {   // a wave per block below 4096 blocks, as the BC1-BC4 block launches
        if (o.bc7enc_perceptual)
            hipLaunchKernelGGL(bc7enc_blocks_wave_kernel<true>, dim3(n), dim3(64), 0, s, (const uint4 *)blocks, n, cf,
                               (uint4 *)dst);
        else
            hipLaunchKernelGGL(bc7enc_blocks_wave_kernel<false>, dim3(n), dim3(64), 0, s, (const uint4 *)blocks, n, cf,
                               (uint4 *)dst);
        return hipGetLastError();
    }
    const uint32_t wg = 256, grid = (n + wg - 1) / wg;
    if (o.bc7enc_perceptual)
        hipLaunchKernelGGL(bc7enc_blocks_kernel<true>, dim3(grid), dim3(wg), 0, s, (const uint4 *)blocks, n, cf,
                           (uint4 *)dst);
    else
        hipLaunchKernelGGL(bc7enc_blocks_kernel<false>, dim3(grid), dim3(wg), 0, s, (const uint4 *)blocks, n, cf,
                           (uint4 *)dst);
    return hipGetLastError();
}

hipError_t launch_bc7enc_blocks_f32(const float *blocks, uint32_t n, const gic_options &o, void *dst, hipStream_t s)
{
    const EncCfg cf = make_cfg(o);
    const uint32_t wg = 256, grid = (n + wg - 1) / wg;
    if (o.bc7enc_perceptual)
        hipLaunchKernelGGL(bc7enc_f32_kernel<true>, dim3(grid), dim3(wg), 0, s, blocks, n, cf, (uint4 *)dst);
    else
        hipLaunchKernelGGL(bc7enc_f32_kernel<false>, dim3(grid), dim3(wg), 0, s, blocks, n, cf, (uint4 *)dst);
    return hipGetLastError();
}

}  // namespace gic

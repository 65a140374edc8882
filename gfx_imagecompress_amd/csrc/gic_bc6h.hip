// gic_bc6h.hip -- BC6H (HDR) block encoder for gfx950 (MI355X).
//
// Algorithm: the reference's BC6HBlockEncoder::CompressBlock at the quality
// Image_CompressAMDBC6H constructs it with (1.0; src/amd_bc6h_body.cpp:1521-1652,
// src/amd_bc6h_compressor.cpp:28) and the HDR_Encode helpers it calls
// (src/amd_hdr_encode.cpp).  Single-precision arithmetic in the reference's
// operation order (-ffp-contract=off, correctly rounded divide / sqrt), so the
// output is bit-identical to the CPU restatement oracle/orc_bc6h.c, which
// states every quirk this file reproduces (the one-region pattern never being
// encoded, the always-unsigned end point decode, QuantizeToInt on the
// unclamped value, ep_shaker_HD's single round on 8-bit codes, ...).
//
// Mapping (a chunk of blocks per pass):
//   K1 k_bc6h_pattern   1 lane / (block, pattern): FindBestPattern (:904-1037)
//                       for the one-region pattern or one of the 32 two-region
//                       shapes -- optQuantAnD_f per subset (4000 rounds with the
//                       stale snapshot; cycles are fast-forwarded exactly),
//                       ep_shaker_HD's 64-corner walk per subset, the clamped
//                       end points and the pattern's CalcShapeError;
//   K2 k_bc6h_encode    1 lane / block: the first strictly smaller pattern
//                       error (shape 31's state when the one-region pattern
//                       wins, :1621-1631), EncodePattern over modes 1..10
//                       (:1351-1488) and SaveDataBlock (:125-454).
// Every per-texel array is held in registers and visited with compile-time
// indices over a 16-bit subset mask (members in texel order = the
// reference's compacted subset order); nothing goes through scratch.

#include <mutex>

#include "gic_common.h"
#include "bc7_tables.h"
#include "bc6h_layout.h"

namespace gic {
namespace bc6h {

constexpr int kPatterns = 33;     // 0 = one region, 1 + s = two-region shape s
constexpr int kF16Max = 0x7bff;   // F16MAX, amd_bc6h_body.hpp:49

__constant__ uint32_t dShape[32];    // BPTC two-subset shapes 0..31, 2 bits per texel
__constant__ uint8_t dAnchor[32];    // anchor texel of subset 1 (g_indexfixups)

struct PatternState {   // FindBestPattern's result for one (block, pattern)
    float err;
    float pad;
    float fep[12];      // fEndPoints[subset][end][channel] after clampF16Max
    uint64_t idx;       // shape_indices per texel, 4 bits each
};

// (int)f with x86 cvttss2si semantics: INT_MIN for NaN and out-of-range
__device__ __forceinline__ int cvt_i32(float f)
{
    return (f >= -2147483648.0f && f < 2147483648.0f) ? (int)f : (int)0x80000000;
}

// IEEE binary16 round to nearest even (the assumed Math_Float2Half; see orc_bc6h.c)
__device__ __forceinline__ uint32_t f2h(float f)
{
    const uint32_t u = __float_as_uint(f);
    const uint32_t sign = (u >> 16) & 0x8000u, ex = (u >> 23) & 0xffu;
    uint32_t man = u & 0x7fffffu;
    if (ex == 0xffu) return sign | 0x7c00u | (man ? 0x200u : 0u);
    const int e = (int)ex - 127 + 15;
    if (e >= 31) return sign | 0x7c00u;
    if (e <= 0) {
        if (e < -10) return sign;
        man |= 0x800000u;
        const int shift = 14 - e;
        uint32_t h = man >> shift;
        const uint32_t rem = man & ((1u << shift) - 1u), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (h & 1u))) h++;
        return sign | h;
    }
    uint32_t h = ((uint32_t)e << 10) | (man >> 13);
    const uint32_t rem = man & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return sign | h;
}

__device__ __forceinline__ int nib(uint64_t v, int t) { return (int)((v >> (4 * t)) & 15u); }
__device__ __forceinline__ uint64_t set_nib(uint64_t v, int t, int x)
{
    return (v & ~(15ull << (4 * t))) | ((uint64_t)(x & 15) << (4 * t));
}

// ---------------------------------------------------------- optQuantAnD_f ---

// quant_AnD_Shell (float), amd_hdr_encode.cpp:1349-1425, over the members of
// `mask`; the fix-up branch keeps the reference's stable qsort via an
// insertion network on (value, member) keys
__device__ __forceinline__ void shell_f(const float prj[16], uint32_t mask, int n, int k, int idx[16])
{
    float m = 0.f, M = 0.f;
    bool first = true;
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if ((mask >> i) & 1u) {
            if (first) {
                m = M = prj[i];
                first = false;
            } else {
                m = m < prj[i] ? m : prj[i];
                M = M > prj[i] ? M : prj[i];
            }
        }
    if (M == m) {
#pragma unroll
        for (int i = 0; i < 16; ++i) idx[i] = 0;
        return;
    }
    const float s = (float)(k - 1) / (M - m);
    float d[16], dm = 0.f, r = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        d[i] = 0.f;
        if ((mask >> i) & 1u) {
            const float v = prj[i] * s;
            const float z = v + 0.5f - m * s;   // not floored (the floor is commented out, :1381)
            idx[i] = cvt_i32(z);
            d[i] = v - z - m * s;
            dm += d[i];
            r += d[i] * d[i];
        }
    }
    if ((float)n * r - dm * dm >= (float)(n - 1) / 4 / 2) {
        dm /= (float)n;
        // members in texel order, then the reference's stable qsort (a_compare:
        // difference sign) as an insertion sort over the first n entries
        float key[16];
        int who[16];
        int q = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            key[i] = 0.f;
            who[i] = 0;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if ((mask >> i) & 1u) {
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    if (j == q) {
                        key[j] = d[i] - dm;
                        who[j] = i;
                    }
                ++q;
            }
#pragma unroll
        for (int a = 1; a < 16; ++a)
#pragma unroll
            for (int b = a; b > 0; --b)
                if (a < n && key[b - 1] - key[b] > 0) {
                    const float tk = key[b];
                    key[b] = key[b - 1];
                    key[b - 1] = tk;
                    const int tw = who[b];
                    who[b] = who[b - 1];
                    who[b - 1] = tw;
                }
        float mm = 0.f, l = 0.f;
        int j = -1;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (i < n) {
                key[i] -= (2.0f * (float)i + 1.0f - (float)n) / 2.0f / (float)n;
                l += key[i];
                if (l < mm) {
                    mm = l;
                    j = i;
                }
            }
        j = (j + 1) % n;
        uint32_t inc = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (i < n && i >= j) inc |= 1u << who[i];
#pragma unroll
        for (int i = 0; i < 16; ++i) idx[i] += (int)((inc >> i) & 1u);
    }
    int mi = 0;
    first = true;
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if ((mask >> i) & 1u) {
            mi = first ? idx[i] : (mi < idx[i] ? mi : idx[i]);
            first = false;
        }
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if ((mask >> i) & 1u) idx[i] -= mi;
}

// eigenVector_d (float), amd_hdr_encode.cpp:1200-1286: p = 5 squarings per
// round, q = 4 rounds (dimension 3); vec untouched when the matrix is zero
__device__ __forceinline__ void eigen_f(const float cov[3][3], float vec[3])
{
    float a[3][3], b[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) a[i][j] = cov[i][j];
    for (int n = 0; n < 4; ++n) {
        float md = 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) md = a[i][i] > md ? a[i][i] : md;
        if (md <= 0) return;
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) a[i][j] /= md;
        for (int m = 0; m < 5; ++m) {
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    float t = 0;
#pragma unroll
                    for (int k = 0; k < 3; ++k) t += a[i][k] * a[k][j];
                    b[i][j] = t;
                }
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) a[i][j] = b[i][j];
        }
    }
    float md = 0;
    int k = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        k = a[i][i] > md ? i : k;
        md = a[i][i] > md ? a[i][i] : md;
    }
    float row[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) row[i] = k == 0 ? a[0][i] : (k == 1 ? a[1][i] : a[2][i]);
    float t = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        t += row[i] * row[i];
        vec[i] = row[i];
    }
    t = sqrtf(t);
    if (t <= 0) return;
#pragma unroll
    for (int i = 0; i < 3; ++i) vec[i] /= t;
}

// per-round state hash for the fast-forward (indices of the members, 4 bits each)
__device__ __forceinline__ uint64_t pack_idx(const int idx[16], uint32_t mask)
{
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if ((mask >> k) & 1u) v |= (uint64_t)(idx[k] & 15) << (4 * k);
    return v;
}

// Iteration cap: optQuantAnD_f's requantisation loop never
// resets try_two (amd_hdr_encode.cpp:1427-1601), so past its exhaustion the
// reference loops until the state is stable -- forever on a cycling state.
// The loop's state is the index vector alone, so once try_two < 0 a Brent
// cycle check (the same in oracle/orc_bc6h.c) stops the loop exactly where a
// revisited state proves the reference never returns (g_nonterm), and a loop
// still running g_iter_cap rounds past the exhaustion within one loop stops
// there (g_iter_hits; the oracle applies the same per-loop cap).  Both stops
// depend only on the loop's starting state, which keeps the 4000-round
// fast-forward below exact.
__device__ int g_iter_cap = 4096;
__device__ unsigned long long g_iter_hits = 0;
__device__ unsigned long long g_nonterm = 0;

// optQuantAnD_f (amd_hdr_encode.cpp:1427-1601), dimension 3, quality 1.0, over
// the members of `mask` (data = din, texel-indexed).  Returns the error; idx
// (texel-indexed) and the GetEndPoints (:1116-1159) end points ep[2][3].
//
// The 4000-round loop compares against the it == 1 snapshot only, so a run
// caught in a cycle that avoids it spins to the end.  The round's state is
// idx after the shell (plus try_two while it is >= 0; once negative its value
// no longer matters); a state recurring after P <= 4 rounds repeats with
// period P and never breaks, so whole periods are skipped -- the final idx is
// the reference's.  The requantisation sweep over the sorted projections is
// the count of thresholds (k + 0.5 - s) t (double, :1532) below each
// projection: the thresholds are non-decreasing in k since t >= 0.
__device__ __forceinline__ float opt_quant_f(const float din[16][3], uint32_t mask, int ncl, int idx[16], float dir[3],
                             float ep[2][3])
{
    const int n = __popc(mask);
    float mean[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        float acc = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if ((mask >> k) & 1u) acc += din[k][i];
        mean[i] = acc / (float)n;
    }
    float cov[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) {
            float acc = 0;
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if ((mask >> k) & 1u) acc += (din[k][i] - mean[i]) * (din[k][j] - mean[j]);
            cov[i][j] = acc;
        }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = i + 1; j < 3; ++j) cov[i][j] = cov[j][i];
    eigen_f(cov, dir);
    float prj[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        prj[k] = 0.f;
        idx[k] = 0;
        if ((mask >> k) & 1u) {
            float acc = 0;
#pragma unroll
            for (int i = 0; i < 3; ++i) acc += (din[k][i] - mean[i]) * dir[i];
            prj[k] = acc;
        }
    }
    uint64_t snap = 0;
    int try_two = 50;
    uint64_t seen[4] = {0, 0, 0, 0};
    int seen_tt[4] = {0, 0, 0, 0};
    bool ff = true;
    for (int it = 0; it < 4000; ++it) {
        if (it >= 2 && ff) {
            const uint64_t cur = pack_idx(idx, mask);
            const int tcls = try_two < 0 ? -1 : try_two;
#pragma unroll
            for (int P = 1; P <= 4; ++P) {
                const int h = (it - P) & 3;
                if (ff && it - P >= 2 && seen[h] == cur && seen_tt[h] == tcls) {
                    it += ((4000 - it) / P) * P;
                    ff = false;
                }
            }
            seen[it & 3] = cur;
            seen_tt[it & 3] = tcls;
            if (it >= 4000) break;
        }
        if (it) {
            bool done;
            uint64_t cyc_saved = 0;
            int cyc_have = 0, cyc_pow = 1, cyc_lam = 0, cyc_rounds = 0;
            do {
                float q = 0, s = 0, t = 0;
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    if ((mask >> k) & 1u) {
                        s += (float)idx[k];
                        t += (float)(idx[k] * idx[k]);
                    }
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    float acc = 0;
#pragma unroll
                    for (int k = 0; k < 16; ++k)
                        if ((mask >> k) & 1u) acc += (din[k][j] - mean[j]) * (float)idx[k];
                    dir[j] = acc;
                    q += dir[j] * dir[j];
                }
                s /= (float)n;
                t = t - s * s * (float)n;
                t = (t == 0.0f ? 0.0f : 1.0f / t);
                q = sqrtf(q);
                t *= q;
                if (q != 0)
#pragma unroll
                    for (int j = 0; j < 3; ++j) dir[j] /= q;
                done = true;
                const double ds = (double)s, dt = (double)t;
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    if ((mask >> k) & 1u) {
                        float acc = 0;
#pragma unroll
                        for (int i = 0; i < 3; ++i) acc += (din[k][i] - mean[i]) * dir[i];
                        prj[k] = acc;
                        int cnt = 0;
                        for (int c = 0; c < ncl - 1; ++c) cnt += ((double)acc > ((double)c + 0.5 - ds) * dt) ? 1 : 0;
                        done = done && cnt == idx[k];
                        idx[k] = cnt;
                    }
                if (!done && try_two < 0) {   // H4: the reference loops until done once try_two < 0
                    const uint64_t st = pack_idx(idx, mask);
                    if (cyc_have && st == cyc_saved) {
                        atomicAdd(&g_nonterm, 1ull);
                        break;
                    }
                    if (++cyc_rounds > g_iter_cap) {
                        atomicAdd(&g_iter_hits, 1ull);
                        break;
                    }
                    if (!cyc_have || ++cyc_lam == cyc_pow) {
                        cyc_saved = st;
                        cyc_have = 1;
                        cyc_pow <<= 1;
                        cyc_lam = 0;
                    }
                }
            } while (!done && try_two--);
            if (it == 1) {
                snap = pack_idx(idx, mask);
            } else if (pack_idx(idx, mask) == snap) {
                break;
            }
        }
        shell_f(prj, mask, n, ncl, idx);
    }
    float q = 0, s = 0, t = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if ((mask >> k) & 1u) {
            s += (float)idx[k];
            t += (float)(idx[k] * idx[k]);
        }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        float acc = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if ((mask >> k) & 1u) acc += (din[k][j] - mean[j]) * (float)idx[k];
        dir[j] = acc;
        q += dir[j] * dir[j];
    }
    s /= (float)n;
    t = t - s * s * (float)n;
    t = (t == 0.0f ? 0.0f : 1.0f / t);
    float err = 0, mn = 65504.0f, mx = 0;
    int mini = -1, maxi = -1;
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if ((mask >> i) & 1u) {
            float o[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                o[j] = mean[j] + dir[j] * t * ((float)idx[i] - s);
                err += (din[i][j] - o[j]) * (din[i][j] - o[j]);
            }
            const float val = o[0] + o[1] + o[2];
            if (mini < 0) mini = maxi = i;   // GetEndPoints' defaults: the first member
            if (val < mn) {
                mn = val;
                mini = i;
            }
            if (val > mx) {
                mx = val;
                maxi = i;
            }
        }
    // end points = the quantised points of the chosen members (recomputed:
    // the same expression gives the same floats)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if (i == mini)
#pragma unroll
            for (int j = 0; j < 3; ++j) ep[0][j] = mean[j] + dir[j] * t * ((float)idx[i] - s);
        if (i == maxi)
#pragma unroll
            for (int j = 0; j < 3; ++j) ep[1][j] = mean[j] + dir[j] * t * ((float)idx[i] - s);
    }
    q = sqrtf(q);
#pragma unroll
    for (int j = 0; j < 3; ++j) dir[j] /= q;
    return err;
}

// ----------------------------------------------------------- ep_shaker_HD ---

__constant__ float kLerpW[5][16] = {
    {0.0f},
    {0.0f, 1.0f},
    {0.0f, 21.0f / 64.0f, 43.0f / 64.0f, 1.0f},
    {0.0f, 9.0f / 64.0f, 18.0f / 64.0f, 27.0f / 64.0f, 37.0f / 64.0f, 46.0f / 64.0f, 55.0f / 64.0f, 1.0f},
    {0.0f, 4.0f / 64.0f, 9.0f / 64.0f, 13.0f / 64.0f, 17.0f / 64.0f, 21.0f / 64.0f, 26.0f / 64.0f, 30.0f / 64.0f,
     34.0f / 64.0f, 38.0f / 64.0f, 43.0f / 64.0f, 47.0f / 64.0f, 51.0f / 64.0f, 55.0f / 64.0f, 60.0f / 64.0f, 1.0f}};

template <int CLOG> struct Lerp;
template <> struct Lerp<0> { __device__ static float w(int) { return 0.0f; } };
template <> struct Lerp<1> { __device__ static float w(int i) { return i ? 1.0f : 0.0f; } };
template <> struct Lerp<2> {
    __device__ static float w(int i)
    {
        return i == 0 ? 0.0f : i == 1 ? 21.0f / 64.0f : i == 2 ? 43.0f / 64.0f : 1.0f;
    }
};
template <> struct Lerp<3> {
    __device__ static float w(int i)
    {
        constexpr float t[8] = {0.0f, 9.0f / 64.0f, 18.0f / 64.0f, 27.0f / 64.0f,
                                37.0f / 64.0f, 46.0f / 64.0f, 55.0f / 64.0f, 1.0f};
        return t[i];
    }
};

// ep_df / expandbits_ with 8-bit codes (amd_hdr_encode.cpp:2098-2111)
__device__ __forceinline__ float ep8(int v) { return (float)(v | (v >> 8)); }

// rampf (USE_NEWRAMP, :2113-2120)
template <int CLOG>
__device__ __forceinline__ float ramp8(float a, float b, int i)
{
    const float ret = floorf(a + Lerp<CLOG>::w(i) * (float)(b - a) + 0.5f);
    return ret > 256.0f ? 255.0f : ret;
}

// ep_shaker_HD (amd_hdr_encode.cpp:2280-2614) for one subset, dimension 3,
// bits {8, 8, 8}, Mi_ = n - 1, CLOG = floor(log2(n)); exactly one round --
// one wavefront per (block, shape, subset).  Lanes t < 16 hold texel t (x[3],
// its quantiser index); the subset's members are visited in texel order with
// readlane broadcasts wherever the reference sums in member order (cluster
// means, the least-squares moments, each corner's error), so every float sum
// is the reference's sequence.  The 64-corner walk runs one corner per lane:
// corner p1's state s is gray(p1), and the walk's first strictly smaller error
// is the minimum of (error bits, p1) -- the errors are sums of squares, so
// their bit patterns order like their values.  (One lane per (block,
// pattern) walking the corners serially held 3 x 8 ramps x 16 texels of
// temporaries: 512 registers, one wave per SIMD, spills.)
__device__ __forceinline__ float rbf(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
__device__ __forceinline__ int rbi(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

struct ShakeOut {        // ep_shaker_HD's result for one (block, shape, subset)
    float err;
    int epo[2][3];      // end point codes
    uint32_t pad;
    uint64_t idx;       // member texels' indices, 4 bits per texel (0 elsewhere)
};

// wave minimum of a non-negative float error and the lowest lane holding it
__device__ __forceinline__ float wave_first_min(float e, int &lane_of)
{
    uint32_t u = __float_as_uint(e);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t v = (uint32_t)__shfl_xor((int)u, o);
        u = v < u ? v : u;
    }
    lane_of = __builtin_ctzll(__ballot(__float_as_uint(e) == u));
    return __uint_as_float(u);
}

template <int CLOG>
__device__ void shake_hd_wave(const float x[3], int idxt, uint32_t mask, ShakeOut &out)
{
    constexpr int NCL = 1 << CLOG;
    const int L = (int)__lane_id();
    const bool mem = L < 16 && ((mask >> L) & 1u);
    const int n = __popc(mask);
    const int Mi_ = n - 1;
    const int f0 = __builtin_ctz(mask);
    // all members equal to the first (exact compares)
    const float y0 = rbf(x[0], f0), y1 = rbf(x[1], f0), y2 = rbf(x[2], f0);
    const bool alls = __all(!mem || (x[0] == y0 && x[1] == y1 && x[2] == y2));
    // index_collapse_kernel (:1688-1713)
    // the set W of the members' indices (< 16): its lowest bit is the minimum
    // and its highest the maximum
    unsigned W = 0;
    for (uint32_t mm = mask; mm; mm &= mm - 1) W |= 1u << (rbi(idxt, __builtin_ctz(mm)) & 15);
    const int mi = __builtin_ctz(W), Mx = 31 - __builtin_clz(W);
    // D = the largest d <= Mx - mi dividing every member's offset idx - mi: the
    // offsets form the 16-bit set V, and lane d tests V against the set of
    // multiples of d -- one ballot instead of a loop of per-lane integer
    // remainders (a ~20-instruction emulated division each)
    const unsigned V = W >> mi;
    unsigned mult = 0;
    if (L >= 2 && L < 16)
        for (int x = 0; x < 16; x += L) mult |= 1u << x;
    const unsigned long long ok = __ballot(L >= 2 && L <= Mx - mi && (V & ~mult) == 0u);
    const int D = ok ? 63 - __builtin_clzll(ok) : 1;
    const int c0 = mem ? (idxt - mi) / D : 0;
    const int Mi = (Mx - mi) / D;
    float err_o = 3.402823466e+38f;
    int idx_new = idxt;
    uint64_t idx_o = 0;
    bool took = false;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) out.epo[i][j] = 0;
    if (Mi == 0) {
        // quant_single_point_d without USE_RAMPS: index 0, end points 0, out 0
        float t = 0;
        if (!alls)
            for (uint32_t mm = mask; mm; mm &= mm - 1) {
                const int u = __builtin_ctz(mm);
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const float v = rbf(x[j], u);
                    t += (v - 0.0f) * (v - 0.0f);
                }
            }
        if (t < err_o) {
            idx_new = 0;
            err_o = t;
        }
    } else {
        // cluster_mean_d_d for this lane's cluster: members in texel order
        float cc[3] = {0.f, 0.f, 0.f};
        {
            float sm[3] = {0.f, 0.f, 0.f};
            int cnt = 0;
            for (uint32_t mm = mask; mm; mm &= mm - 1) {
                const int u = __builtin_ctz(mm);
                const bool same = rbi(c0, u) == c0;
                cnt += same ? 1 : 0;
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const float v = rbf(x[j], u);
                    sm[j] = same ? sm[j] + v : sm[j];
                }
            }
            if (mem)
#pragma unroll
                for (int j = 0; j < 3; ++j) cc[j] = floorf(sm[j] / (float)cnt + 0.5f);
        }
        // The least-squares sums of an expansion ck = c0 * q + p are float sums of
        // integers below 2^24 in magnitude (|cc| <= 0x7c00, Mi_ <= 15, <= 16
        // members), so every partial sum is exact and they equal integer
        // polynomials in (q, p) over the subset's moments N, S1 = sum c0,
        // S2 = sum c0^2, C0 = sum cc, C1 = sum c0 * cc.
        int S1 = 0, S2 = 0, C0[3] = {0, 0, 0}, C1[3] = {0, 0, 0};
        for (uint32_t mm = mask; mm; mm &= mm - 1) {
            const int u = __builtin_ctz(mm);
            const int cu = rbi(c0, u);
            S1 += cu;
            S2 += cu * cu;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int c = (int)rbf(cc[j], u);
                C0[j] += c;
                C1[j] += cu * c;
            }
        }
        const int s = L ^ (L >> 1);   // the walk's state after step p1 = L
        float err_2 = 3.402823466e+38f;
        uint64_t idx_2 = 0;
        int epo_2[2][3] = {{0, 0, 0}, {0, 0, 0}};
        for (int q = 1; q * Mi <= Mi_; q++)
            for (int p = 0; p <= Mi_ - q * Mi; p++) {
                // least squares on the rounded cluster means (:2377-2437)
                const int sc = q * S1 + p * n, sc2 = q * q * S2 + 2 * p * q * S1 + p * p * n;
                const float im00 = (float)(Mi_ * Mi_ * n - 2 * Mi_ * sc + sc2), im01 = (float)(Mi_ * sc - sc2),
                            im11 = (float)sc2;
                float rp[2][3];
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const int r1 = q * C1[j] + p * C0[j];
                    rp[0][j] = (float)(Mi_ * C0[j] - r1);
                    rp[1][j] = (float)r1;
                }
                const float dd = im00 * im11 - im01 * im01;
                const float i10 = im00;
                const float a00 = im11 / dd, a11 = i10 / dd, a01 = -im01 / dd;
                float epd[2][3][2], eq[2][3][2];
#pragma unroll
                for (int j = 0; j < 3; j++) {
                    const float e0 = (a00 * rp[0][j] + a01 * rp[1][j]) * (float)Mi_;
                    const float e1 = (a01 * rp[0][j] + a11 * rp[1][j]) * (float)Mi_;
                    epd[0][j][0] = epd[0][j][1] = e0;
                    epd[1][j][0] = epd[1][j][1] = e1;
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const int lim = (int)(255u - (uint32_t)cvt_i32(epd[i][j][1]));
                        epd[i][j][1] += (float)(lim < 1 ? lim : 1);
                    }
#pragma unroll
                    for (int i = 0; i < 2; ++i)
#pragma unroll
                        for (int c = 0; c < 2; ++c) eq[i][j][c] = ep8(cvt_i32(epd[i][j][c]));
                }
                // corner s of the 64-corner walk (:2476-2549): per channel j, end
                // point 0's candidate (s >> 2j) & 1 and end point 1's (s >> 2j+1) & 1
                float R[3][NCL];
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const float a = ((s >> (2 * j)) & 1) ? eq[0][j][1] : eq[0][j][0];
                    const float b = ((s >> (2 * j + 1)) & 1) ? eq[1][j][1] : eq[1][j][0];
#pragma unroll
                    for (int c = 0; c < NCL; ++c) R[j][c] = ramp8<CLOG>(a, b, c);
                }
                // Exact cut: the partial sums only grow (non-negative terms), so once
                // every corner's partial error has reached err_2 this expansion
                // cannot change the outcome (it needs err_1 < err_2) and its walk
                // is abandoned.
                float err_0 = 0;
                uint64_t idx_0 = 0;
                bool cut = false;
                int k = 0;
                for (uint32_t mm = mask; mm; mm &= mm - 1, ++k) {
                    if ((k & 1) == 0 && k && __all(err_0 >= err_2)) {
                        cut = true;
                        break;
                    }
                    const int i = __builtin_ctz(mm);
                    const float d0 = rbf(x[0], i), d1 = rbf(x[1], i), d2 = rbf(x[2], i);
                    int ci = 0;
                    float cmin = 3.402823466e+38f;
#pragma unroll
                    for (int c = 0; c < NCL; c++) {
                        const float r0 = R[0][c] - d0, r1 = R[1][c] - d1, r2 = R[2][c] - d2;
                        float t_ = 0.f;
                        t_ += r0 * r0;
                        t_ += r1 * r1;
                        t_ += r2 * r2;
                        if (t_ < cmin) {
                            cmin = t_;
                            ci = c;
                        }
                    }
                    idx_0 |= (uint64_t)ci << (4 * i);
                    err_0 += cmin;
                }
                if (cut) continue;
                int w;
                const float err_1 = wave_first_min(err_0, w);
                if (err_1 < err_2) {
                    err_2 = err_1;
                    const uint32_t lo = (uint32_t)rbi((int)(uint32_t)idx_0, w), hi = (uint32_t)rbi((int)(uint32_t)(idx_0 >> 32), w);
                    idx_2 = ((uint64_t)hi << 32) | lo;
                    const int s1 = w ^ (w >> 1);
#pragma unroll
                    for (int j = 0; j < 3; j++) {
                        epo_2[0][j] = cvt_i32(epd[0][j][(s1 >> (2 * j)) & 1]);
                        epo_2[1][j] = cvt_i32(epd[1][j][(s1 >> (2 * j + 1)) & 1]);
                    }
                }
            }
        if (err_2 < err_o) {
            took = true;
            idx_o = idx_2;
#pragma unroll
            for (int j = 0; j < 3; j++) {
                out.epo[0][j] = epo_2[0][j];
                out.epo[1][j] = epo_2[1][j];
            }
            err_o = err_2;
        }
    }
    if (!took) {   // the members' indices as they stand (quantiser's, or 0 from the single point)
        uint64_t v = 0;
        for (uint32_t mm = mask; mm; mm &= mm - 1) {
            const int u = __builtin_ctz(mm);
            v |= (uint64_t)(rbi(idx_new, u) & 15) << (4 * u);
        }
        idx_o = v;
    }
    out.err = err_o;
    out.idx = idx_o;
    out.pad = 0;
}

// ---------------------------------------------------------- block loading ---

struct Src {
    const float *blocks;   // float RGBA blocks (64 per block), or null: the image
    Geometry g;
    int force_alpha_one;
};

// CompressBlock's texel conversion (:1539-1573)
__device__ __forceinline__ void load_din(const Src &src, uint32_t b, int is_signed, float din[16][3])
{
    float blk[64];
    if (src.blocks) {
        const float4 *p = reinterpret_cast<const float4 *>(src.blocks + (size_t)b * 64);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float4 v = p[i];
            blk[i * 4 + 0] = v.x;
            blk[i * 4 + 1] = v.y;
            blk[i * 4 + 2] = v.z;
            blk[i * 4 + 3] = v.w;
        }
    } else {
        uint32_t slice, by, bx;
        block_coords(src.g, b, slice, by, bx);
        load_block(src.g, slice, by, bx, src.force_alpha_one != 0, blk);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float v = blk[i * 4 + c];
            if ((double)v < 0.00001)
                din[i][c] = is_signed ? (float)-(int)f2h(fabsf(v / 1.0f)) : 0.0f;
            else
                din[i][c] = (float)(int)f2h(v / 1.0f);
        }
}

__device__ __forceinline__ uint32_t subset_mask(int shape, int sub)
{
    if (shape < 0) return sub ? 0u : 0xFFFFu;
    const uint32_t w = dShape[shape];
    uint32_t m = 0;
#pragma unroll
    for (int t = 0; t < 16; ++t) m |= (((w >> (2 * t)) & 3u) == (uint32_t)sub ? 1u : 0u) << t;
    return m;
}

__device__ __forceinline__ float clamp_f16(float v, int is_signed)
{
    if (is_signed) {
        if (v < -kF16Max) return -kF16Max;
        if (v > kF16Max) return kF16Max;
    } else {
        if (v < 0.0) return 0;
        if (v > kF16Max) return kF16Max;
    }
    return v;
}

// lerpf (:66-81) for denominators 7 and 15
__device__ __forceinline__ float lerp_pal(float a, float b, int i, int denom)
{
    const int w7[8] = {0, 9, 18, 27, 37, 46, 55, 64};
    const int w15[16] = {0, 4, 9, 13, 17, 21, 26, 30, 34, 38, 43, 47, 51, 55, 60, 64};
    int wa = 0, wb = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int v = denom == 7 ? (k < 8 ? w7[k] : 0) : w15[k];
        wa = k == denom - i ? v : wa;
        wb = k == i ? v : wb;
    }
    return (a * (float)wa + b * (float)wb) / 64.0f;
}

// palitizeEndPointsF (:707-758): region 1 = 16 entries of subset 0, region 2
// = 8 entries per subset (pal[sub * 8 + i])
template <int REGION>
__device__ __forceinline__ void palette(const float fep[12], float pal[16][3])
{
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            if (REGION == 1)
                pal[i][c] = lerp_pal(fep[c], fep[3 + c], i, 15);
            else
                pal[i][c] = lerp_pal(fep[(i >> 3) * 6 + c], fep[(i >> 3) * 6 + 3 + c], i & 7, 7);
        }
}

// CalcShapeError (:783-836): per texel, the palette scan of its subset from
// entry 0 while the sum of absolute differences does not increase
template <int REGION>
__device__ __forceinline__ float shape_error(const float din[16][3], uint32_t m1, const float pal[16][3])
{
    constexpr int MAXP = REGION == 1 ? 16 : 8;
    float total = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const bool sub = REGION == 2 && ((m1 >> i) & 1u);
        float best = 0.f;
        bool go = true;
#pragma unroll
        for (int j = 0; j < MAXP; j++) {
            const float p0 = sub ? pal[8 + (j & 7)][0] : pal[j][0], p1 = sub ? pal[8 + (j & 7)][1] : pal[j][1],
                        p2 = sub ? pal[8 + (j & 7)][2] : pal[j][2];
            const float er = fabsf(din[i][0] - p0) + fabsf(din[i][1] - p1) + fabsf(din[i][2] - p2);
            if (j == 0) {
                best = er;
            } else if (go && best > 0) {
                if (er <= best)
                    best = er;
                else
                    go = false;
            }
        }
        total += best;
    }
    return total;
}

// FindBestPattern (:904-1037) in four launches per chunk:
//   K0 k_bc6h_prep    lane / block: CompressBlock's texel conversion (f2h) into
//                     the din workspace (every later kernel reads it);
//   K1 k_bc6h_quant   lane / (block, pattern): optQuantAnD_f per subset;
//   K2 k_bc6h_shake   wave / (block, two-region shape, subset): ep_shaker_HD;
//   K3 k_bc6h_final   lane / (block, pattern): the shaker's result where it is
//                     better, clampF16Max, the pattern's CalcShapeError.
struct QuantState {     // optQuantAnD_f's results for one (block, pattern)
    float err;          // summed over the subsets in subset order
    float pad;
    uint64_t idx;       // indices of both subsets, 4 bits per texel
    float ep[2][2][3];  // GetEndPoints per subset
};

__global__ void __launch_bounds__(256) k_bc6h_prep(Src src, uint32_t first, uint32_t n, int is_signed,
                                                   float *__restrict__ din_ws)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n) return;
    float din[16][3];
    load_din(src, first + b, is_signed, din);
    float *o = din_ws + (size_t)b * 48;
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int c = 0; c < 3; ++c) o[i * 3 + c] = din[i][c];
}

__device__ __forceinline__ void read_din(const float *__restrict__ din_ws, uint32_t b, float din[16][3])
{
    const float4 *p = reinterpret_cast<const float4 *>(din_ws + (size_t)b * 48);
    float v[48];
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        const float4 w = p[k];
        v[4 * k] = w.x;
        v[4 * k + 1] = w.y;
        v[4 * k + 2] = w.z;
        v[4 * k + 3] = w.w;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int c = 0; c < 3; ++c) din[i][c] = v[i * 3 + c];
}

__global__ void __launch_bounds__(256) k_bc6h_quant(uint32_t n, const float *__restrict__ din_ws,
                                                    QuantState *__restrict__ qs)
{
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t b = gid / kPatterns;
    const int pat = (int)(gid % kPatterns);
    if (b >= n) return;
    float din[16][3];
    read_din(din_ws, b, din);
    const int shape = pat - 1;
    const int ns = shape >= 0 ? 2 : 1, ncl = shape >= 0 ? 8 : 16;
    float dir[3] = {0.f, 0.f, 0.f};
    QuantState q;
    q.err = 0.0f;
    q.pad = 0.0f;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int c = 0; c < 3; ++c) q.ep[s][e][c] = 0.f;
    int qidx[16];
    uint64_t idx0 = 0;
    const uint32_t masks[2] = {subset_mask(shape, 0), subset_mask(shape, 1)};
    for (int s = 0; s < ns; ++s) {
        q.err += opt_quant_f(din, masks[s], ncl, qidx, dir, q.ep[s]);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if ((masks[s] >> k) & 1u) idx0 = set_nib(idx0, k, qidx[k]);
    }
    q.idx = idx0;
    qs[(size_t)b * kPatterns + pat] = q;
}

// USE_SHAKERHD at quality 1.0 > 0.80 (:960-1025): every two-region shape's
// subsets are shaken from the quantiser's indices
// 6 waves/SIMD (70 VGPRs): 69.2 -> 66.8 ms unsigned, 320 -> 308 ms signed per
// 1024^2 against the unconstrained 88-VGPR build, same blocks
__global__ void __launch_bounds__(256, 6) k_bc6h_shake(uint32_t n, const float *__restrict__ din_ws,
                                                    const QuantState *__restrict__ qs, ShakeOut *__restrict__ so)
{
    // wave-uniform by construction; readfirstlane lets the compiler see it
    const uint32_t wid = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t b = wid >> 6;
    const int shape = (int)((wid >> 1) & 31u), sub = (int)(wid & 1u);
    if (b >= n) return;   // whole waves
    const int L = (int)__lane_id();
    float x[3] = {0.f, 0.f, 0.f};
    if (L < 16)
#pragma unroll
        for (int c = 0; c < 3; ++c) x[c] = din_ws[(size_t)b * 48 + L * 3 + c];
    const uint64_t qi = qs[(size_t)b * kPatterns + 1 + shape].idx;
    const int idxt = L < 16 ? nib(qi, L) : 0;
    const uint32_t mask = subset_mask(shape, sub);
    const int nm = __popc(mask);
    ShakeOut out;
    if (nm >= 8)
        shake_hd_wave<3>(x, idxt, mask, out);
    else if (nm >= 4)
        shake_hd_wave<2>(x, idxt, mask, out);
    else if (nm >= 2)
        shake_hd_wave<1>(x, idxt, mask, out);
    else
        shake_hd_wave<0>(x, idxt, mask, out);
    if (L == 0) so[((size_t)b * 32 + shape) * 2 + sub] = out;
}

__global__ void __launch_bounds__(256) k_bc6h_final(uint32_t n, int is_signed, const float *__restrict__ din_ws,
                                                    const QuantState *__restrict__ qs, const ShakeOut *__restrict__ so,
                                                    PatternState *__restrict__ ws)
{
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t b = gid / kPatterns;
    const int pat = (int)(gid % kPatterns);
    if (b >= n) return;
    const QuantState q = qs[(size_t)b * kPatterns + pat];
    const int shape = pat - 1;
    const int ns = shape >= 0 ? 2 : 1;
    PatternState st;
    st.pad = 0.f;
    uint64_t idx = q.idx;
    bool shaker = false;
    int epo[2][2][3] = {};
    if (shape >= 0) {
        const ShakeOut s0 = so[((size_t)b * 32 + shape) * 2], s1 = so[((size_t)b * 32 + shape) * 2 + 1];
        float err1 = 0.0f;
        err1 += s0.err;
        err1 += s1.err;
        if (q.err > err1) {
            shaker = true;
            idx = s0.idx | s1.idx;   // disjoint member nibbles
        }
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                epo[0][e][c] = s0.epo[e][c];
                epo[1][e][c] = s1.epo[e][c];
            }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int c = 0; c < 3; ++c)
                st.fep[(s * 2 + e) * 3 + c] =
                    clamp_f16(shaker && s < ns ? (float)epo[s][e][c] : q.ep[s][e][c], is_signed);
    st.idx = idx;
    float din[16][3];
    read_din(din_ws, b, din);
    float pal[16][3];
    if (shape >= 0) {
        palette<2>(st.fep, pal);
        st.err = shape_error<2>(din, subset_mask(shape, 1), pal);
    } else {
        palette<1>(st.fep, pal);
        st.err = shape_error<1>(din, 0u, pal);
    }
    ws[(size_t)b * kPatterns + pat] = st;
}

// ---------------------------------------------------------- EncodePattern ---

struct ModePart {
    int nbits, prec[3], transformed, index_prec, mode;
};
// ModePartition (amd_bc6h_body.hpp:157-178), modes 1..10
__constant__ ModePart kMP[11] = {
    {0, {0, 0, 0}, 0, 0, 0},     {10, {5, 5, 5}, 1, 3, 0x00}, {7, {6, 6, 6}, 1, 3, 0x01}, {11, {5, 4, 4}, 1, 3, 0x02},
    {11, {4, 5, 4}, 1, 3, 0x06}, {11, {4, 4, 5}, 1, 3, 0x0a}, {9, {5, 5, 5}, 1, 3, 0x0e}, {8, {6, 5, 5}, 1, 3, 0x12},
    {8, {5, 6, 5}, 1, 3, 0x16},  {8, {5, 5, 6}, 1, 3, 0x1a},  {6, {6, 6, 6}, 0, 3, 0x1e},
};

__device__ __forceinline__ int maskn(int n) { return (1 << n) - 1; }
__device__ __forceinline__ int sign_extend(int w, int tbits)
{
    return ((w & (1 << (tbits - 1))) ? (int)(~0u << tbits) : 0) | w;
}

// QuantizeToInt (amd_hdr_encode.cpp:83-115) of (short)(int)v
__device__ __forceinline__ int quantize_to_int(float v, int prec, int is_signed)
{
    const short value = (short)cvt_i32(v);
    if (prec <= 1) return 0;
    bool neg = false;
    const int ivalue = value;
    if (is_signed) {
        neg = value < 0;
        prec--;
    }
    int bias = (prec > 10 && prec != 16) ? ((1 << (prec - 11)) - 1) : 0;
    bias = (prec == 16) ? 15 : bias;
    const int q = (int)(((long long)ivalue * (1ll << prec) + bias) / (kF16Max + 1));
    return neg ? -q : q;
}

__device__ __forceinline__ bool is_overflow(int v, int nbit)
{
    return !(v >= -(1 << (nbit - 1)) && v <= (1 << (nbit - 1)) - 1);
}

// TransformEndPoints (amd_bc6h_body.cpp:598-660), two regions
__device__ bool transform_ep(const ModePart &mp, const int ie[12], int oe[12])
{
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const int p = mp.prec[i], pm = maskn(p);
        oe[i] = ie[i] & maskn(mp.nbits);
        if (mp.transformed) {
#pragma unroll
            for (int r = 1; r < 4; ++r) {
                const int d = ie[r * 3 + i] - ie[i];
                if (is_overflow(d, p)) return false;
                oe[r * 3 + i] = d & pm;
            }
        } else {
#pragma unroll
            for (int r = 1; r < 4; ++r) oe[r * 3 + i] = ie[r * 3 + i] & pm;
        }
    }
    return true;
}

// endpts_fit (:493-507) with decompress_endpts (:458-490)
__device__ bool endpoints_fit(const ModePart &mp, const int orig[12], const int comp[12], int is_signed)
{
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        int un[4];
        if (mp.transformed) {
            un[0] = is_signed ? sign_extend(comp[i], mp.index_prec) : comp[i];
#pragma unroll
            for (int r = 1; r < 4; ++r) {
                const int t = (sign_extend(comp[r * 3 + i], mp.prec[i]) + comp[i]) & maskn(mp.nbits);
                un[r] = is_signed ? sign_extend(t, mp.nbits) : t;
            }
        } else {
            un[0] = is_signed ? sign_extend(comp[i], mp.nbits) : comp[i];
#pragma unroll
            for (int r = 1; r < 4; ++r) un[r] = is_signed ? sign_extend(comp[r * 3 + i], mp.prec[i]) : comp[r * 3 + i];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) ok = ok && orig[r * 3 + i] == un[r];
    }
    return ok;
}

// Unquantize (:117-150) + finish_unquantizeF16 (:1039-1049), unsigned
__device__ __forceinline__ float unq_f16(int comp, int bits)
{
    int unq;
    if (bits >= 15)
        unq = comp;
    else if (comp == 0)
        unq = 0;
    else if (comp == ((1 << bits) - 1))
        unq = 0xFFFF;
    else
        unq = ((comp << 16) + 0x8000) >> bits;
    return (float)((unq * 31) >> 6);
}

// decompress_endpoints2 (:1134-1252), the unsigned branches (issigned is never set)
__device__ void decode_ep2(const ModePart &mp, const int oe[12], float out[12])
{
#pragma unroll
    for (int i = 0; i < 3; i++) {
        int o[4];
        o[0] = oe[i];
#pragma unroll
        for (int r = 1; r < 4; ++r)
            o[r] = mp.transformed ? (sign_extend(oe[r * 3 + i], mp.prec[i]) + oe[i]) & maskn(mp.nbits) : oe[r * 3 + i];
#pragma unroll
        for (int r = 0; r < 4; ++r) out[r * 3 + i] = unq_f16(o[r], mp.nbits);
    }
}

// SwapIndices (:555-581): subset 0's anchor is texel 0, subset 1's dAnchor[shape]
__device__ void swap_indices(int ie[12], uint64_t &idx, int shape, uint32_t m1)
{
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const int at = s ? (int)dAnchor[shape] : 0;
        if (nib(idx, at) & 4) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int t = ie[s * 6 + c];
                ie[s * 6 + c] = ie[s * 6 + 3 + c];
                ie[s * 6 + 3 + c] = t;
            }
            const uint32_t ms = s ? m1 : (~m1 & 0xFFFFu);
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if ((ms >> k) & 1u) idx = set_nib(idx, k, 7 - nib(idx, k));
        }
    }
}

// SaveDataBlock field layout (amd_bc6h_body.cpp:132-364): per mode, (first
// bit, bits, field, shift); fields rw gw bw rx gx bx ry gy by rz gz bz, 12 = mode
struct BitField {
    uint8_t start, bits, field, shift;
};
enum { RW, GW, BW, RX, GX, BX, RY, GY, BY, RZ, GZ, BZ, MV };
__constant__ BitField kLayout[11][24] = {
    {{0, 0, 0, 0}},
    {{0, 2, MV, 0},   {2, 1, GY, 4},   {3, 1, BY, 4},   {4, 1, BZ, 4},   {5, 10, RW, 0}, {15, 10, GW, 0},
     {25, 10, BW, 0}, {35, 5, RX, 0},  {40, 1, GZ, 4},  {41, 4, GY, 0},  {45, 5, GX, 0}, {50, 1, BZ, 0},
     {51, 4, GZ, 0},  {55, 5, BX, 0},  {60, 1, BZ, 1},  {61, 4, BY, 0},  {65, 5, RY, 0}, {70, 1, BZ, 2},
     {71, 5, RZ, 0},  {76, 1, BZ, 3},  {0, 0, 0, 0}},
    {{0, 2, MV, 0},   {2, 1, GY, 5},   {3, 1, GZ, 4},   {4, 1, GZ, 5},   {5, 7, RW, 0},  {12, 1, BZ, 0},
     {13, 1, BZ, 1},  {14, 1, BY, 4},  {15, 7, GW, 0},  {22, 1, BY, 5},  {23, 1, BZ, 2}, {24, 1, GY, 4},
     {25, 7, BW, 0},  {32, 1, BZ, 3},  {33, 1, BZ, 5},  {34, 1, BZ, 4},  {35, 6, RX, 0}, {41, 4, GY, 0},
     {45, 6, GX, 0},  {51, 4, GZ, 0},  {55, 6, BX, 0},  {61, 4, BY, 0},  {65, 6, RY, 0}, {71, 6, RZ, 0}},
    {{0, 5, MV, 0},   {5, 10, RW, 0},  {15, 10, GW, 0}, {25, 10, BW, 0}, {35, 5, RX, 0}, {40, 1, RW, 10},
     {41, 4, GY, 0},  {45, 4, GX, 0},  {49, 1, GW, 10}, {50, 1, BZ, 0},  {51, 4, GZ, 0}, {55, 4, BX, 0},
     {59, 1, BW, 10}, {60, 1, BZ, 1},  {61, 4, BY, 0},  {65, 5, RY, 0},  {70, 1, BZ, 2}, {71, 5, RZ, 0},
     {76, 1, BZ, 3},  {0, 0, 0, 0}},
    {{0, 5, MV, 0},   {5, 10, RW, 0},  {15, 10, GW, 0}, {25, 10, BW, 0}, {35, 4, RX, 0}, {39, 1, RW, 10},
     {40, 1, GZ, 4},  {41, 4, GY, 0},  {45, 5, GX, 0},  {50, 1, GW, 10}, {51, 4, GZ, 0}, {55, 4, BX, 0},
     {59, 1, BW, 10}, {60, 1, BZ, 1},  {61, 4, BY, 0},  {65, 4, RY, 0},  {69, 1, BZ, 0}, {70, 1, BZ, 2},
     {71, 4, RZ, 0},  {75, 1, GY, 4},  {76, 1, BZ, 3},  {0, 0, 0, 0}},
    {{0, 5, MV, 0},   {5, 10, RW, 0},  {15, 10, GW, 0}, {25, 10, BW, 0}, {35, 4, RX, 0}, {39, 1, RW, 10},
     {40, 1, BY, 4},  {41, 4, GY, 0},  {45, 4, GX, 0},  {49, 1, GW, 10}, {50, 1, BZ, 0}, {51, 4, GZ, 0},
     {55, 5, BX, 0},  {60, 1, BW, 10}, {61, 4, BY, 0},  {65, 4, RY, 0},  {69, 1, BZ, 1}, {70, 1, BZ, 2},
     {71, 4, RZ, 0},  {75, 1, BZ, 4},  {76, 1, BZ, 3},  {0, 0, 0, 0}},
    {{0, 5, MV, 0},   {5, 9, RW, 0},   {14, 1, BY, 4},  {15, 9, GW, 0},  {24, 1, GY, 4}, {25, 9, BW, 0},
     {34, 1, BZ, 4},  {35, 5, RX, 0},  {40, 1, GZ, 4},  {41, 4, GY, 0},  {45, 5, GX, 0}, {50, 1, BZ, 0},
     {51, 4, GZ, 0},  {55, 5, BX, 0},  {60, 1, BZ, 1},  {61, 4, BY, 0},  {65, 5, RY, 0}, {70, 1, BZ, 2},
     {71, 5, RZ, 0},  {76, 1, BZ, 3},  {0, 0, 0, 0}},
    {{0, 5, MV, 0},   {5, 8, RW, 0},   {13, 1, GZ, 4},  {14, 1, BY, 4},  {15, 8, GW, 0}, {23, 1, BZ, 2},
     {24, 1, GY, 4},  {25, 8, BW, 0},  {33, 1, BZ, 3},  {34, 1, BZ, 4},  {35, 6, RX, 0}, {41, 4, GY, 0},
     {45, 5, GX, 0},  {50, 1, BZ, 0},  {51, 4, GZ, 0},  {55, 5, BX, 0},  {60, 1, BZ, 1}, {61, 4, BY, 0},
     {65, 6, RY, 0},  {71, 6, RZ, 0},  {0, 0, 0, 0}},
    {{0, 5, MV, 0},   {5, 8, RW, 0},   {13, 1, BZ, 0},  {14, 1, BY, 4},  {15, 8, GW, 0}, {23, 1, GY, 5},
     {24, 1, GY, 4},  {25, 8, BW, 0},  {33, 1, GZ, 5},  {34, 1, BZ, 4},  {35, 5, RX, 0}, {40, 1, GZ, 4},
     {41, 4, GY, 0},  {45, 6, GX, 0},  {51, 4, GZ, 0},  {55, 5, BX, 0},  {60, 1, BZ, 1}, {61, 4, BY, 0},
     {65, 5, RY, 0},  {70, 1, BZ, 2},  {71, 5, RZ, 0},  {76, 1, BZ, 3},  {0, 0, 0, 0}},
    {{0, 5, MV, 0},   {5, 8, RW, 0},   {13, 1, BZ, 1},  {14, 1, BY, 4},  {15, 8, GW, 0}, {23, 1, BY, 5},
     {24, 1, GY, 4},  {25, 8, BW, 0},  {33, 1, BZ, 5},  {34, 1, BZ, 4},  {35, 5, RX, 0}, {40, 1, GZ, 4},
     {41, 4, GY, 0},  {45, 5, GX, 0},  {50, 1, BZ, 0},  {51, 4, GZ, 0},  {55, 6, BX, 0}, {61, 4, BY, 0},
     {65, 5, RY, 0},  {70, 1, BZ, 2},  {71, 5, RZ, 0},  {76, 1, BZ, 3},  {0, 0, 0, 0}},
    {{0, 5, MV, 0},   {5, 6, RW, 0},   {11, 1, GZ, 4},  {12, 1, BZ, 0},  {13, 1, BZ, 1}, {14, 1, BY, 4},
     {15, 6, GW, 0},  {21, 1, GY, 5},  {22, 1, BY, 5},  {23, 1, BZ, 2},  {24, 1, GY, 4}, {25, 6, BW, 0},
     {31, 1, GZ, 5},  {32, 1, BZ, 3},  {33, 1, BZ, 5},  {34, 1, BZ, 4},  {35, 6, RX, 0}, {41, 4, GY, 0},
     {45, 6, GX, 0},  {51, 4, GZ, 0},  {55, 6, BX, 0},  {61, 4, BY, 0},  {65, 6, RY, 0}, {71, 6, RZ, 0}},
};

// BitHeader::setvalue (:88-100) into a 128-bit block held as 4 words
__device__ __forceinline__ void set_bits(uint32_t w[4], int start, int bits, int value, int shift)
{
    for (int k = 0; k < bits; ++k) {
        const int pos = start + k;
        const uint32_t bit = ((uint32_t)value >> (shift + k)) & 1u;
        const int wi = pos >> 5, bi = pos & 31;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (q == wi) w[q] = (w[q] & ~(1u << bi)) | (bit << bi);
    }
}

__device__ void save_block(int mode, int shape, const int oe[12], uint64_t idx, uint32_t m1, uint4 *out)
{
    // the reference's field names: w = [0][0], x = [0][1], y = [1][0], z = [1][1]
    int f[13];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        f[RW + c] = oe[c];
        f[RX + c] = oe[3 + c];
        f[RY + c] = oe[6 + c];
        f[RZ + c] = oe[9 + c];
    }
    f[MV] = kMP[mode].mode;
    uint32_t w[4] = {0, 0, 0, 0};
    for (int k = 0; k < 24; ++k) {
        const BitField bf = kLayout[mode][k];
        if (!bf.bits) break;
        int v = 0;
#pragma unroll
        for (int q = 0; q < 13; ++q) v = q == bf.field ? f[q] : v;
        set_bits(w, bf.start, bf.bits, v, bf.shift);
    }
    set_bits(w, 77, 5, shape, 0);
    const int anc = dAnchor[shape];
    int start = 82, nb = 2;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if (i) {
            start += nb;
            nb = anc == i ? 2 : 3;
        }
        set_bits(w, start, nb, nib(idx, i), 0);
    }
    (void)m1;
    *out = make_uint4(w[0], w[1], w[2], w[3]);
}

// ReIndexShapef (:838-902): each texel's nearest palette entry of its subset
// (first strictly smaller sum of absolute differences)
__device__ __forceinline__ uint64_t reindex(const float din[16][3], const float pal[16][3], uint32_t m1)
{
    uint64_t idx = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const bool sub = (m1 >> i) & 1u;
        float best = 3.402823466e+38f;
        int bi = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const float p0 = sub ? pal[8 + j][0] : pal[j][0], p1 = sub ? pal[8 + j][1] : pal[j][1],
                        p2 = sub ? pal[8 + j][2] : pal[j][2];
            const float e = fabsf(din[i][0] - p0) + fabsf(din[i][1] - p1) + fabsf(din[i][2] - p2);
            if (e < best) {
                best = e;
                bi = j;
            }
        }
        idx |= (uint64_t)bi << (4 * i);
    }
    return idx;
}

__constant__ uint32_t kRedBlock[4] = {0x00007bc2u, 0x00000000u, 0x0003e000u, 0x00000000u};

// K2: pattern selection (:1593-1632), EncodePattern (:1351-1488), SaveDataBlock
__global__ void __launch_bounds__(256) k_bc6h_encode(uint32_t first, uint32_t n, int is_signed,
                                                     const float *__restrict__ din_ws,
                                                     const PatternState *__restrict__ ws, uint4 *__restrict__ dst,
                                                     double *__restrict__ err_out)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n) return;
    const PatternState *pst = ws + (size_t)b * kPatterns;
    float best_err = pst[0].err;
    int best = -1;
    for (int s = 0; s < 32; ++s) {
        const float e = pst[1 + s].err;
        if (e < best_err) {
            best_err = e;
            best = s;
        }
    }
    const int shape = best >= 0 ? best : 31;   // nothing restored when the one-region pattern wins
    const PatternState st = pst[1 + shape];
    float din[16][3];
    read_din(din_ws, b, din);
    const uint32_t m1 = subset_mask(shape, 1);
    float error = best_err, best_e = 3.402823466e+38f;
    int best_fit = 0, numfits = 0;
    int best_q[12];
    uint64_t best_idx = 0;
#pragma unroll
    for (int k = 0; k < 12; ++k) best_q[k] = 0;
    for (int m = 1; m <= 10; ++m) {
        const ModePart mp = kMP[m];
        int ie[12], oe[12];
        uint64_t idx = st.idx;
#pragma unroll
        for (int k = 0; k < 12; ++k) ie[k] = quantize_to_int(st.fep[k], mp.nbits, is_signed);
        swap_indices(ie, idx, shape, m1);
        if (!transform_ep(mp, ie, oe)) continue;
        if (!endpoints_fit(mp, ie, oe, is_signed)) continue;
        numfits++;
        float dec[12];
        decode_ep2(mp, oe, dec);
        float pal[16][3];
        palette<2>(dec, pal);
        if (!is_signed) idx = reindex(din, pal, m1);
        const float e = shape_error<2>(din, m1, pal);
        if (e < best_e) {
            bool tf = true;
            if (!is_signed) {
#pragma unroll
                for (int k = 0; k < 12; ++k) ie[k] = quantize_to_int(dec[k], mp.nbits, 0);
                swap_indices(ie, idx, shape, m1);
                tf = transform_ep(mp, ie, oe);
            }
            if (tf) {
                best_fit = m;
                best_e = e;
                error = e;
#pragma unroll
                for (int k = 0; k < 12; ++k) best_q[k] = oe[k];
                best_idx = idx;
            }
        }
    }
    if (numfits > 0 && best_fit > 0) {
        save_block(best_fit, shape, best_q, best_idx, m1, dst + first + b);
    } else {
        dst[first + b] = make_uint4(kRedBlock[0], kRedBlock[1], kRedBlock[2], kRedBlock[3]);
    }
    if (err_out) err_out[first + b] = (double)error;
}

// --------------------------------------------------------------- decoder ---
//
// gic_hip_decode_bc6h: BC6H blocks back to RGBA16F texels (alpha 1.0), one lane
// per block, from the format description -- the header layouts of
// bc6h_layout.h (tools/gen_bc6h_layout.py, a transcription independent of the
// encoder's kLayout), endpoint sign extension and inverse transform,
// unquantisation, the 3/4-bit weights and the 31/64 (unsigned) or 31/32
// (signed) finish.  Reserved modes decode to zero.

__constant__ int kWeights3[8] = {0, 9, 18, 27, 37, 46, 55, 64};
__constant__ int kWeights4[16] = {0, 4, 9, 13, 17, 21, 26, 30, 34, 38, 43, 47, 51, 55, 60, 64};

__device__ __forceinline__ int dec_sext(int x, int bits) { return (x << (32 - bits)) >> (32 - bits); }

__device__ __forceinline__ int dec_unq(int x, int bits, bool is_signed)
{
    if (!is_signed) {
        if (bits >= 15) return x;
        if (x == 0) return 0;
        if (x == (1 << bits) - 1) return 0xFFFF;
        return ((x << 16) + 0x8000) >> bits;
    }
    if (bits >= 16) return x;
    const bool neg = x < 0;
    const int a = neg ? -x : x;
    int u;
    if (a == 0)
        u = 0;
    else if (a >= (1 << (bits - 1)) - 1)
        u = 0x7FFF;
    else
        u = ((a << 15) + 0x4000) >> (bits - 1);
    return neg ? -u : u;
}

__device__ __forceinline__ uint32_t dec_finish(int v, bool is_signed)
{
    if (!is_signed) return (uint32_t)((v * 31) >> 6);
    const int h = v < 0 ? -(((-v) * 31) >> 5) : (v * 31) >> 5;
    return h < 0 ? (0x8000u | (uint32_t)(-h)) : (uint32_t)h;
}

__global__ void __launch_bounds__(256) k_bc6h_decode(const uint8_t *__restrict__ blocks, uint32_t width, uint32_t height,
                                                     uint32_t slices, int is_signed, uint16_t *__restrict__ out,
                                                     size_t row_pitch)
{
    const uint32_t bx = (width + 3) / 4, by = (height + 3) / 4;
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= bx * by * slices) return;
    const uint32_t sl = id / (bx * by), r = id % (bx * by), y0 = (r / bx) * 4, x0 = (r % bx) * 4;
    const uint4 w = reinterpret_cast<const uint4 *>(blocks)[id];
    const uint64_t lo = (uint64_t)w.x | ((uint64_t)w.y << 32), hi = (uint64_t)w.z | ((uint64_t)w.w << 32);
    auto bit = [&](uint32_t p) -> uint32_t { return (uint32_t)((p < 64 ? lo >> p : hi >> (p - 64)) & 1u); };
    auto take = [&](uint32_t &p, uint32_t n) -> uint32_t {
        uint32_t v = 0;
        for (uint32_t k = 0; k < n; ++k) v |= bit(p + k) << k;
        p += n;
        return v;
    };
    int mode = -1;
    const uint32_t m2 = w.x & 3u, m5 = w.x & 31u;
    for (int m = 0; m < 14; ++m) {
        const ModeDesc &d = kDecModes[m];
        if ((d.mode_bits == 2 && m2 == d.value) || (d.mode_bits == 5 && m2 >= 2 && m5 == d.value)) {
            mode = m;
            break;
        }
    }
    uint16_t tex[16][3];
    if (mode < 0) {
        for (int t = 0; t < 16; ++t) tex[t][0] = tex[t][1] = tex[t][2] = 0;
    } else {
        const ModeDesc d = kDecModes[mode];
        uint32_t p = d.mode_bits;
        int f[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int e = 0; e < d.n; ++e) {
            const int code = kDecLayout[mode][e];
            f[code >> 4] |= (int)take(p, 1) << (code & 15);
        }
        const int regions = d.regions, nends = 2 * regions;
        const uint32_t part = regions == 2 ? take(p, 5) : 0u;
        const int epb = d.ep_bits;
        int ep[4][3];
        for (int e = 0; e < 4; ++e)
            for (int c = 0; c < 3; ++c) ep[e][c] = f[e * 3 + c];
        for (int c = 0; c < 3; ++c) {
            if (is_signed) ep[0][c] = dec_sext(ep[0][c], epb);
            for (int e = 1; e < nends; ++e) {
                if (d.transformed) {
                    const int v = (ep[0][c] + dec_sext(ep[e][c], d.delta_bits[c])) & ((1 << epb) - 1);
                    ep[e][c] = is_signed ? dec_sext(v, epb) : v;
                } else if (is_signed) {
                    ep[e][c] = dec_sext(ep[e][c], epb);
                }
            }
        }
        int unq[4][3];
        for (int e = 0; e < nends; ++e)
            for (int c = 0; c < 3; ++c) unq[e][c] = dec_unq(ep[e][c], epb, is_signed != 0);
        const uint32_t shape = regions == 2 ? dShape[part] : 0u;
        const uint32_t anc = regions == 2 ? dAnchor[part] : 0u;
        const uint32_t ib = regions == 2 ? 3 : 4;
        for (int t = 0; t < 16; ++t) {
            const bool anchor = t == 0 || (regions == 2 && (uint32_t)t == anc);
            const uint32_t idx = take(p, anchor ? ib - 1 : ib);
            const int wgt = ib == 3 ? kWeights3[idx] : kWeights4[idx];
            const int rg = (int)((shape >> (2 * t)) & 3u);
            for (int c = 0; c < 3; ++c) {
                const int v = ((64 - wgt) * unq[2 * rg][c] + wgt * unq[2 * rg + 1][c] + 32) >> 6;
                tex[t][c] = (uint16_t)dec_finish(v, is_signed != 0);
            }
        }
    }
    for (int t = 0; t < 16; ++t) {
        const uint32_t x = x0 + (t & 3), y = y0 + (t >> 2);
        if (x >= width || y >= height) continue;
        uint16_t *o = (uint16_t *)((uint8_t *)out + ((size_t)sl * height + y) * row_pitch) + (size_t)x * 4;
        o[0] = tex[t][0];
        o[1] = tex[t][1];
        o[2] = tex[t][2];
        o[3] = 0x3C00;   // 1.0
    }
}

// ------------------------------------------------------------------ host ---

constexpr uint32_t kChunk = 1u << 16;

static hipError_t upload_tables()
{
    static bool done[64] = {};   // per device, guarded by the caller's lock
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    if (done[dev]) return hipSuccess;
    uint32_t shp[32];
    uint8_t anc[32];
    for (int s = 0; s < 32; ++s) {
        shp[s] = kBc7Shape2[s];
        anc[s] = kBc7Anchor2[s];
    }
    e = hipMemcpyToSymbol(HIP_SYMBOL(dShape), shp, sizeof(shp));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(dAnchor), anc, sizeof(anc));
    if (e == hipSuccess) done[dev] = true;
    return e;
}

}  // namespace bc6h

static std::mutex g_bc6h_lock;

// n blocks from float RGBA blocks (blocks != null) or from the image g, in
// passes of kChunk blocks with a stream-ordered pattern workspace
static hipError_t bc6h_run(const float *blocks, const Geometry *g, uint32_t n, int is_signed, int force_alpha_one,
                           void *dst, double *err, hipStream_t s)
{
    using namespace bc6h;
    {
        std::lock_guard<std::mutex> lk(g_bc6h_lock);
        const hipError_t e = upload_tables();
        if (e != hipSuccess) return e;
    }
    const uint32_t chunk = n < kChunk ? n : kChunk;
    // one allocation: din, quantiser states, shaker outputs, pattern states
    const size_t sz_din = ((size_t)chunk * 48 * sizeof(float) + 255) & ~(size_t)255;
    const size_t sz_q = ((size_t)chunk * kPatterns * sizeof(QuantState) + 255) & ~(size_t)255;
    const size_t sz_s = ((size_t)chunk * 64 * sizeof(ShakeOut) + 255) & ~(size_t)255;
    const size_t sz_p = (size_t)chunk * kPatterns * sizeof(PatternState);
    char *mem = nullptr;
    hipError_t e = hipMallocAsync((void **)&mem, sz_din + sz_q + sz_s + sz_p, s);
    if (e != hipSuccess) return e;
    float *din = (float *)mem;
    QuantState *qs = (QuantState *)(mem + sz_din);
    ShakeOut *so = (ShakeOut *)(mem + sz_din + sz_q);
    PatternState *ws = (PatternState *)(mem + sz_din + sz_q + sz_s);
    Src src;
    src.blocks = blocks;
    if (g) src.g = *g;
    src.force_alpha_one = force_alpha_one;
    for (uint32_t first = 0; first < n; first += chunk) {
        const uint32_t m = (n - first) < chunk ? (n - first) : chunk;
        const uint64_t nl = (uint64_t)m * kPatterns, nw = (uint64_t)m * 64 * 64;
        hipLaunchKernelGGL(k_bc6h_prep, dim3((m + 255) / 256), dim3(256), 0, s, src, first, m, is_signed, din);
        hipLaunchKernelGGL(k_bc6h_quant, dim3((uint32_t)((nl + 255) / 256)), dim3(256), 0, s, m, (const float *)din,
                           qs);
        hipLaunchKernelGGL(k_bc6h_shake, dim3((uint32_t)((nw + 255) / 256)), dim3(256), 0, s, m, (const float *)din,
                           (const QuantState *)qs, so);
        hipLaunchKernelGGL(k_bc6h_final, dim3((uint32_t)((nl + 255) / 256)), dim3(256), 0, s, m, is_signed,
                           (const float *)din, (const QuantState *)qs, (const ShakeOut *)so, ws);
        hipLaunchKernelGGL(k_bc6h_encode, dim3((m + 255) / 256), dim3(256), 0, s, first, m, is_signed,
                           (const float *)din, (const PatternState *)ws, (uint4 *)dst, err);
        e = hipGetLastError();
        if (e != hipSuccess) break;
    }
    const hipError_t ef = hipFreeAsync(mem, s);
    return e != hipSuccess ? e : ef;
}

hipError_t bc6h_nonterm(unsigned long long *n, int reset)
{
    hipError_t e = hipMemcpyFromSymbol(n, HIP_SYMBOL(bc6h::g_nonterm), sizeof(*n));
    if (e == hipSuccess && reset) {
        const unsigned long long z = 0;
        e = hipMemcpyToSymbol(HIP_SYMBOL(bc6h::g_nonterm), &z, sizeof(z));
    }
    return e;
}

hipError_t bc6h_iter_cap(int cap, unsigned long long *hits, int reset)
{
    hipError_t e = hipSuccess;
    if (hits) e = hipMemcpyFromSymbol(hits, HIP_SYMBOL(bc6h::g_iter_hits), sizeof(*hits));
    if (e == hipSuccess && reset) {
        const unsigned long long z = 0;
        e = hipMemcpyToSymbol(HIP_SYMBOL(bc6h::g_iter_hits), &z, sizeof(z));
    }
    if (e == hipSuccess && cap >= 0) e = hipMemcpyToSymbol(HIP_SYMBOL(bc6h::g_iter_cap), &cap, sizeof(cap));
    return e;
}

hipError_t launch_bc6h_decode(const uint8_t *blocks, uint32_t width, uint32_t height, uint32_t slices, int is_signed,
                              uint16_t *out, size_t row_pitch, hipStream_t s)
{
    using namespace bc6h;
    {
        std::lock_guard<std::mutex> lk(g_bc6h_lock);
        const hipError_t e = upload_tables();
        if (e != hipSuccess) return e;
    }
    const uint64_t n = (uint64_t)((width + 3) / 4) * ((height + 3) / 4) * slices;
    hipLaunchKernelGGL(k_bc6h_decode, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, blocks, width, height, slices,
                       is_signed, out, row_pitch);
    return hipGetLastError();
}

hipError_t launch_bc6h_blocks(const float *blocks, uint32_t n, int is_signed, void *dst, double *err, hipStream_t s)
{
    return bc6h_run(blocks, nullptr, n, is_signed, 0, dst, err, s);
}

hipError_t launch_bc6h_image(const Geometry &g, int is_signed, int force_alpha_one, void *dst, double *err,
                             hipStream_t s)
{
    return bc6h_run(nullptr, &g, g.total, is_signed, force_alpha_one, dst, err, s);
}

}  // namespace gic

/*
 * orc_bc6h.c -- CPU restatement of the reference's BC6H block encoder.
 *
 * TEST INFRASTRUCTURE ONLY (see bcn_oracle.h): the parity checker for the HIP
 * BC6H kernels in gfx_imagecompress_amd/csrc/gic_bc6h.hip.
 *
 * Follows BC6HBlockEncoder::CompressBlock (src/amd_bc6h_body.cpp:1521-1652)
 * with the encoder constructed by Image_CompressAMDBC6H
 * (src/amd_bc6h_compressor.cpp:28: quality 1.0), and the HDR_Encode helpers
 * it calls (src/amd_hdr_encode.cpp).  Arithmetic is single precision in the
 * reference's operation order (build with -ffp-contract=off); the
 * requantisation threshold test of optQuantAnD_f is in double, as written.
 *
 * What the reference does, stated here (each point cites its lines):
 *  - texels become half-float bit patterns held in floats: Math_Float2Half
 *    (al2o3_cmath, un-vendored) is taken as IEEE binary16 round-to-nearest-
 *    even -- the conversion is PARITY-UNPINNED, as is the whole BC6H path (no
 *    reference fixture holds BC6H output);
 *  - FindBestPattern (:904-1037) for the one-region pattern and the 32
 *    two-region shapes: optQuantAnD_f per subset (16 or 8 clusters,
 *    MAX_TRY * quality = 4000 rounds with the stale i == 1 snapshot, as the
 *    BC7 quantiser), then -- USE_SHAKERHD is defined (:116) and quality > 0.8
 *    -- ep_shaker_HD per subset of the two-region shapes with bits {8, 8, 8}
 *    and Mi_ = entryCount - 1 (:977-986); end points from the quantiser's min /
 *    max points (GetEndPoints) or the shaker's codes, clamped to [0, 0x7bff]
 *    (signed: +-0x7bff), error = CalcShapeError (absolute differences);
 *  - CompressBlock keeps the first strictly smaller pattern error; when the
 *    one-region pattern is never beaten, nothing is restored (:1621-1631) and
 *    the state left is shape 31's, so EncodePattern always sees region 2:
 *    modes 1..10 only, the one-region modes 11..14 are unreachable;
 *  - EncodePattern (:1351-1488) tries modes 1..10: quantise (QuantizeToInt,
 *    which shifts the unclamped value), anchor swap, transform with overflow
 *    checks, lossless-fit check, decode (decompress_endpoints2 -- `issigned`
 *    is never set, :1140, so always the unsigned decode), palette, re-index
 *    (unsigned only), CalcShapeError; the first strictly smaller error wins,
 *    re-quantised from the decoded end points (unsigned);
 *  - no fitting mode, or no mode whose re-quantisation transforms, leaves
 *    m_mode 0 and writes the reference's red block (:1639-1645);
 *  - SaveDataBlock (:125-454) bit layout per mode, shape index at bit 77,
 *    indices from bit 82 with the anchor's high bit dropped.
 * x86 conversions of out-of-range floats to int give INT_MIN; that is made
 * explicit (cvt_i32) so the GPU can reproduce it.
 */
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "bcn_oracle.h"
#include "bc7_tables.h"

#define F16MAX 0x7bff
#define HALF_MAX_F 65504.0f   /* HALF_MAX 0x1.ffcp15, amd_hdr_encode.cpp:37 */

/* --------------------------------------------------------------- helpers --- */

/* (int)f as x86 cvttss2si: truncation, INT_MIN for NaN and out-of-range */
static int cvt_i32(float f)
{
    if (!(f >= -2147483648.0f && f < 2147483648.0f)) return INT_MIN;
    return (int)f;
}

/* IEEE binary16 from binary32, round to nearest even (the assumed
 * Math_Float2Half); returns the 16-bit pattern */
uint16_t orc_float_to_half(float f)
{
    uint32_t u;
    memcpy(&u, &f, 4);
    const uint32_t sign = (u >> 16) & 0x8000u;
    const uint32_t ex = (u >> 23) & 0xffu;
    uint32_t man = u & 0x7fffffu;
    if (ex == 0xffu) return (uint16_t)(sign | 0x7c00u | (man ? 0x200u : 0u));
    const int e = (int)ex - 127 + 15;
    if (e >= 31) return (uint16_t)(sign | 0x7c00u);
    if (e <= 0) {
        if (e < -10) return (uint16_t)sign;
        man |= 0x800000u;
        const int shift = 14 - e;
        uint32_t h = man >> shift;
        const uint32_t rem = man & ((1u << shift) - 1u), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (h & 1u))) h++;
        return (uint16_t)(sign | h);
    }
    uint32_t h = ((uint32_t)e << 10) | (man >> 13);
    const uint32_t rem = man & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;   /* may carry into the exponent: correct */
    return (uint16_t)(sign | h);
}

static int shape2_of(int shape, int t) { return (int)((kBc7Shape2[shape] >> (2 * t)) & 3u); }

/* g_indexfixups (amd_bc6h_body.hpp:210-220) = the BPTC anchor of subset 1;
 * g_Region2FixUp (:194-204) = its position among subset 1's texels */
static int anchor_texel(int shape) { return kBc7Anchor2[shape]; }
static int anchor_pos(int shape)
{
    int p = 0;
    for (int t = 0; t < anchor_texel(shape); ++t) p += shape2_of(shape, t);
    return p;
}

int orc_bc6h_anchor(int shape, int *pos)
{
    *pos = anchor_pos(shape);
    return anchor_texel(shape);
}

/* ModePartition (amd_bc6h_body.hpp:157-178): nbits, prec[3], transformed,
 * modebits, IndexPrec, mode value, lowestPrec */
typedef struct {
    int nbits, prec[3], transformed, modebits, index_prec, mode, lowest;
} mode_part;
static const mode_part kMP[15] = {
    {0, {0, 0, 0}, 0, 0, 0, 0x00, 0},       {10, {5, 5, 5}, 1, 2, 3, 0x00, 31}, {7, {6, 6, 6}, 1, 2, 3, 0x01, 248},
    {11, {5, 4, 4}, 1, 5, 3, 0x02, 15},     {11, {4, 5, 4}, 1, 5, 3, 0x06, 15}, {11, {4, 4, 5}, 1, 5, 3, 0x0a, 15},
    {9, {5, 5, 5}, 1, 5, 3, 0x0e, 62},      {8, {6, 5, 5}, 1, 5, 3, 0x12, 124}, {8, {5, 6, 5}, 1, 5, 3, 0x16, 124},
    {8, {5, 5, 6}, 1, 5, 3, 0x1a, 124},     {6, {6, 6, 6}, 0, 5, 3, 0x1e, 496}, {10, {10, 10, 10}, 0, 5, 4, 0x03, 31},
    {11, {9, 9, 9}, 1, 5, 4, 0x07, 15},     {12, {8, 8, 8}, 1, 5, 4, 0x0b, 7},  {16, {4, 4, 4}, 1, 5, 4, 0x0f, 1},
};

#define MASKN(n) ((1 << (n)) - 1)
static int sign_extend(int w, int tbits)   /* SIGN_EXTEND, amd_bc6h_body.hpp:72 */
{
    return ((w & (1 << (tbits - 1))) ? (int)(~0u << tbits) : 0) | w;
}

/* lerpf, amd_hdr_encode.cpp:66-81 (denominators 7 and 15 here) */
static const int kW3[8] = {0, 9, 18, 27, 37, 46, 55, 64};
static const int kW4[16] = {0, 4, 9, 13, 17, 21, 26, 30, 34, 38, 43, 47, 51, 55, 60, 64};
static float lerp_pal(float a, float b, int i, int denom)
{
    const int *w = denom == 7 ? kW3 : kW4;
    return (a * (float)w[denom - i] + b * (float)w[i]) / 64.0f;
}

/* ------------------------------------------------------- optQuantAnD_f --- */

typedef struct {
    float d;
    int i;
} keyf;

/* qsort with a_compare (difference sign), glibc's stable merge sort */
static void stable_sort_f(keyf *a, int n)
{
    for (int i = 1; i < n; ++i) {
        keyf t = a[i];
        int j = i - 1;
        while (j >= 0 && a[j].d - t.d > 0) {
            a[j + 1] = a[j];
            --j;
        }
        a[j + 1] = t;
    }
}

/* eigenVector_d (float), amd_hdr_encode.cpp:1200-1286: p squarings per round,
 * q rounds, p = floor(log2((FLT_MAX_EXP - 2) / ceil(log2(3)))) = 5, q = 4 */
static int ev_p(void)
{
    const int dimension = 3;
    int p = (int)floorf(logf((FLT_MAX_EXP - 2) / ceilf(logf((float)dimension) / logf(2.0f))) / logf(2.0f));
    return p > 0 ? p : 1;
}

static void eigen_f(float cov[4][4], float vec[4])
{
    float c[2][4][4];
    const int dim = 3;
    for (int i = 0; i < dim; ++i)
        for (int j = 0; j < dim; ++j) c[0][i][j] = cov[i][j];
    const int p = ev_p(), q = (20 + p - 1) / p;
    int l = 0;
    for (int n = 0; n < q; ++n) {
        float md = 0;
        for (int i = 0; i < dim; ++i) md = c[l][i][i] > md ? c[l][i][i] : md;
        if (md <= 0) return;   /* vec left as the caller had it */
        for (int i = 0; i < dim; ++i)
            for (int j = 0; j < dim; ++j) c[l][i][j] /= md;
        for (int m = 0; m < p; ++m) {
            for (int i = 0; i < dim; ++i)
                for (int j = 0; j < dim; ++j) {
                    float t = 0;
                    for (int k = 0; k < dim; ++k) t += c[l][i][k] * c[l][k][j];
                    c[1 - l][i][j] = t;
                }
            l = 1 - l;
        }
    }
    float md = 0;
    int k = 0;
    for (int i = 0; i < dim; ++i) {
        k = c[l][i][i] > md ? i : k;
        md = c[l][i][i] > md ? c[l][i][i] : md;
    }
    float t = 0;
    for (int i = 0; i < dim; ++i) {
        t += c[l][k][i] * c[l][k][i];
        vec[i] = c[l][k][i];
    }
    t = sqrtf(t);
    if (t <= 0) return;
    for (int i = 0; i < dim; ++i) vec[i] /= t;
}

static void project_f(float data[][4], int n, const float *v, float *out)
{
    for (int k = 0; k < n; ++k) {
        out[k] = 0;
        for (int i = 0; i < 3; ++i) out[k] += data[k][i] * v[i];
    }
}

/* quant_AnD_Shell (float), amd_hdr_encode.cpp:1349-1425: z keeps the unfloored
 * value (the floor is commented out), so d = v - z - m*s ~ -0.5 */
static void shell_f(const float *v_, int k, int n, int *idx)
{
    float v[16], z[16];
    keyf d[16];
    float m = v_[0], M = v_[0], dm = 0.f, r = 0;
    for (int i = 1; i < n; ++i) {
        m = m < v_[i] ? m : v_[i];
        M = M > v_[i] ? M : v_[i];
    }
    if (M == m) {
        for (int i = 0; i < n; ++i) idx[i] = 0;
        return;
    }
    const float s = (float)(k - 1) / (M - m);
    for (int i = 0; i < n; ++i) {
        v[i] = v_[i] * s;
        z[i] = v[i] + 0.5f - m * s;
        idx[i] = cvt_i32(z[i]);
        d[i].d = v[i] - z[i] - m * s;
        d[i].i = i;
        dm += d[i].d;
        r += d[i].d * d[i].d;
    }
    if (n * r - dm * dm >= (float)(n - 1) / 4 / 2) {
        dm /= (float)n;
        for (int i = 0; i < n; ++i) d[i].d -= dm;
        stable_sort_f(d, n);
        for (int i = 0; i < n; ++i) d[i].d -= (2.0f * (float)i + 1.0f - (float)n) / 2.0f / (float)n;
        float mm = 0.f, l = 0.f;
        int j = -1;
        for (int i = 0; i < n; ++i) {
            l += d[i].d;
            if (l < mm) {
                mm = l;
                j = i;
            }
        }
        j = (j + 1) % n;
        for (int i = j; i < n; ++i) idx[d[i].i]++;
    }
    int mi = idx[0];
    for (int i = 1; i < n; ++i) mi = mi < idx[i] ? mi : idx[i];
    for (int i = 0; i < n; ++i) idx[i] -= mi;
}

/* Once try_two has run negative the reference's `while (!done && try_two--)`
 * loops until a fixed point -- forever on a cycling state.  The loop's state is
 * the index vector alone, so a revisited state proves non-termination: a Brent
 * cycle check stops the loop there (the reference never returns for such a
 * block), and a loop still running g_cap rounds past the exhaustion within
 * one loop stops too.  The GPU (gic_bc6h.hip opt_quant_f) applies the same two
 * stops in the same order, so both agree on every block. */
static int g_cap = 4096;
static unsigned long long g_nonterm_loops, g_cap_loops;
void orc_bc6h_set_cap(int cap) { g_cap = cap < 0 ? 4096 : cap; }
void orc_bc6h_h4_counts(unsigned long long *nonterm, unsigned long long *capped)
{
    if (nonterm) *nonterm = __atomic_load_n(&g_nonterm_loops, __ATOMIC_RELAXED);
    if (capped) *capped = __atomic_load_n(&g_cap_loops, __ATOMIC_RELAXED);
}

/* optQuantAnD_f, amd_hdr_encode.cpp:1427-1601 (dimension 3, quality 1.0) */
static float opt_quant_f(float data[][4], int n, int ncl, int *index, float out[][4], float dir[4])
{
    int snap[16], order[16];
    float cen[16][4], mean[4], cov[4][4], prj[16];
    float s, t;
    int try_two = 50;
    const int max_try = (int)(4000 * 1.0f);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < 3; ++j) cen[i][j] = data[i][j];
    for (int i = 0; i < 3; ++i) {   /* centerInPlace_d :1178-1198 */
        mean[i] = 0;
        for (int k = 0; k < n; ++k) mean[i] += cen[k][i];
    }
    if (n) {
        for (int i = 0; i < 3; ++i) {
            mean[i] /= (float)n;
            for (int k = 0; k < n; ++k) cen[k][i] -= mean[i];
        }
    }
    for (int i = 0; i < 3; ++i)   /* covariance_d :1161-1176 */
        for (int j = 0; j <= i; ++j) {
            cov[i][j] = 0;
            for (int k = 0; k < n; ++k) cov[i][j] += cen[k][i] * cen[k][j];
        }
    for (int i = 0; i < 3; ++i)
        for (int j = i + 1; j < 3; ++j) cov[i][j] = cov[j][i];
    if (n == 0) return 0.f;
    eigen_f(cov, dir);
    project_f(cen, n, dir, prj);
    for (int it = 0; it < max_try; ++it) {
        if (it) {
            int done;
            uint64_t cyc_saved = 0;
            int cyc_have = 0, cyc_pow = 1, cyc_lam = 0, cyc_rounds = 0;
            do {
                float q = 0;
                s = t = 0;
                for (int k = 0; k < n; ++k) {
                    s += index[k];
                    t += index[k] * index[k];
                }
                for (int j = 0; j < 3; ++j) {
                    dir[j] = 0;
                    for (int k = 0; k < n; ++k) dir[j] += cen[k][j] * index[k];
                    q += dir[j] * dir[j];
                }
                s /= (float)n;
                t = t - s * s * (float)n;
                t = (t == 0.0f ? 0.0f : 1.0f / t);
                q = sqrtf(q);
                t *= q;
                if (q != 0)
                    for (int j = 0; j < 3; ++j) dir[j] /= q;
                project_f(cen, n, dir, prj);
                {   /* sortProjection :1315-1327 */
                    keyf w[16];
                    for (int i = 0; i < n; ++i) {
                        w[i].i = i;
                        w[i].d = prj[i];
                    }
                    stable_sort_f(w, n);
                    for (int i = 0; i < n; ++i) order[i] = w[i].i;
                }
                int nidx[16], k = 0;
                for (int j = 0; j < n; ++j) {
                    /* (k + 0.5 - s) * t is evaluated in double (:1532) */
                    while ((double)prj[order[j]] > ((double)k + 0.5 - (double)s) * (double)t && k < ncl - 1) k++;
                    nidx[order[j]] = k;
                }
                done = 1;
                uint64_t st = 0;
                for (int j = 0; j < n; ++j) {
                    done = (done && (nidx[j] == index[j]));
                    index[j] = nidx[j];
                    st |= (uint64_t)(nidx[j] & 15) << (4 * j);
                }
                if (!done && try_two < 0) {
                    if (cyc_have && st == cyc_saved) {   /* a cycle: the reference never returns */
                        __atomic_fetch_add(&g_nonterm_loops, 1, __ATOMIC_RELAXED);
                        break;
                    }
                    if (++cyc_rounds > g_cap) {
                        __atomic_fetch_add(&g_cap_loops, 1, __ATOMIC_RELAXED);
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
                for (int j = 0; j < n; ++j) snap[j] = index[j];
            } else {
                /* :1547-1557: compares against the it == 1 snapshot, never refreshed */
                done = 1;
                for (int j = 0; j < n; ++j) done = (done && (snap[j] == index[j]));
                if (done) break;
            }
        }
        shell_f(prj, ncl, n, index);
    }
    float q = 0;
    s = t = 0;
    for (int k = 0; k < n; ++k) {
        s += index[k];
        t += index[k] * index[k];
    }
    for (int j = 0; j < 3; ++j) {
        dir[j] = 0;
        for (int k = 0; k < n; ++k) dir[j] += cen[k][j] * index[k];
        q += dir[j] * dir[j];
    }
    s /= (float)n;
    t = t - s * s * (float)n;
    t = (t == 0.0 ? 0.0f : 1.0f / t);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < 3; ++j) out[i][j] = mean[j] + dir[j] * t * ((float)index[i] - s);
    q = sqrtf(q);
    for (int j = 0; j < 3; ++j) dir[j] /= q;
    float e = 0;   /* totalError_d :1329-1338 */
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < 3; ++j) e += (data[i][j] - out[i][j]) * (data[i][j] - out[i][j]);
    return e;
}

/* ------------------------------------------------------- ep_shaker_HD --- */

static const float kLerpW[5][16] = {   /* rampLerpWeights, amd_hdr_encode.cpp:1613-1621 */
    {0.0f},
    {0.0f, 1.0f},
    {0.0f, 21.0f / 64.0f, 43.0f / 64.0f, 1.0f},
    {0.0f, 9.0f / 64.0f, 18.0f / 64.0f, 27.0f / 64.0f, 37.0f / 64.0f, 46.0f / 64.0f, 55.0f / 64.0f, 1.0f},
    {0.0f, 4.0f / 64.0f, 9.0f / 64.0f, 13.0f / 64.0f, 17.0f / 64.0f, 21.0f / 64.0f, 26.0f / 64.0f, 30.0f / 64.0f,
     34.0f / 64.0f, 38.0f / 64.0f, 43.0f / 64.0f, 47.0f / 64.0f, 51.0f / 64.0f, 55.0f / 64.0f, 60.0f / 64.0f, 1.0f}};

/* ep_df / expandbits_ with 8 bits (bits {8, 8, 8}): v | v >> 8 (:2098-2111) */
static float ep8(int v) { return (float)(v | (v >> 8)); }   /* v << 0 == v (also for v < 0) */

/* rampf (USE_NEWRAMP, :2113-2120) with 8-bit codes; clog = log2 of the ramp size */
static float ramp8(int clog, int p1, int p2, int i)
{
    const float a = ep8(p1), b = ep8(p2);
    const float ret = floorf(a + kLerpW[clog][i] * (float)(b - a) + 0.5f);
    if (ret > 256.0f) return 255.0f;
    return ret;
}

/* ep_shaker_HD, amd_hdr_encode.cpp:2280-2614, dimension 3, bits {8, 8, 8}
 * (use_par 0), Mi_ = numEntries - 1.  maxTry starts at 1 and is decremented
 * before the loop test, so exactly one round runs. */
#ifdef ORC_STATS
unsigned long long orc_bc6h_stats[4];
#endif
static float shaker_hd(float data[][4], int n, int *index_, int epo_code[2][4])
{
    const int Mi_ = n - 1;
    int clog = 0;
    for (int i = Mi_ + 1; i >>= 1;) clog++;
    const int ncl = 1 << clog;
    int index[16];
    for (int k = 0; k < n; ++k) index[k] = index_[k];
    float err_o = FLT_MAX;
    int alls = 1;   /* all_same_d :1629-1638 */
    for (int i = 1; i < n; ++i)
        for (int j = 0; j < 3; ++j) alls = alls && (data[0][j] == data[i][j]);
    /* index_collapse_kernel :1688-1713 */
    {
        int mi = index[0], Mx = index[0];
        for (int k = 1; k < n; ++k) {
            mi = mi < index[k] ? mi : index[k];
            Mx = Mx > index[k] ? Mx : index[k];
        }
        int D = 1;
        for (int d = 2; d <= Mx - mi; d++) {
            int k;
            for (k = 0; k < n; k++)
                if ((index[k] - mi) % d != 0) break;
            if (k >= n) D = d;
        }
        for (int k = 0; k < n; k++) index[k] = (index[k] - mi) / D;
    }
    int Mi = index[0];
    for (int k = 0; k < n; ++k) Mi = Mi > index[k] ? Mi : index[k];
    if (Mi == 0) {
        /* quant_single_point_d (:1903-2094) without USE_RAMPS: every candidate
         * costs 0, so index 0 and end points 0 win; out = 0 */
        float t = 0;
        if (!alls)
            for (int i = 0; i < n; ++i)
                for (int j = 0; j < 3; ++j) t += (data[i][j] - 0.0f) * (data[i][j] - 0.0f);
        if (t < err_o) {
            for (int k = 0; k < n; ++k) index_[k] = 0;
            for (int j = 0; j < 3; ++j) epo_code[0][j] = epo_code[1][j] = 0;
            err_o = t;
        }
        return err_o;
    }
    int p0 = -1, q0 = -1;
    float err_2 = FLT_MAX;
    int idx_2[16], epo_2[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#ifdef ORC_STATS
    /* instrumentation build only: shaker calls, expansions, texel-corner work */
    {
        extern unsigned long long orc_bc6h_stats[4];
        __atomic_fetch_add(&orc_bc6h_stats[0], 1ull, __ATOMIC_RELAXED);
        unsigned long long ne = 0;
        for (int q = 1; q * Mi <= Mi_; q++) ne += (unsigned long long)(Mi_ - q * Mi + 1);
        __atomic_fetch_add(&orc_bc6h_stats[1], ne, __ATOMIC_RELAXED);
        __atomic_fetch_add(&orc_bc6h_stats[2], ne * 64ull * (unsigned long long)n, __ATOMIC_RELAXED);
        __atomic_fetch_add(&orc_bc6h_stats[3], Mi == 1 ? 1ull : 0ull, __ATOMIC_RELAXED);
    }
#endif
    for (int q = 1; q * Mi <= Mi_; q++)
        for (int p = 0; p <= Mi_ - q * Mi; p++) {
            int cidx[16];
            for (int k = 0; k < n; k++) cidx[k] = index[k] * q + p;
            /* cluster_mean_d_d :1649-1674, rounded */
            float cc[16][4];
            int cnt[16], comp[16], ncomp = 0;
            for (int i = 0; i < n; i++)
                for (int j = 0; j < 3; j++) {
                    cc[cidx[i]][j] = 0;
                    cnt[cidx[i]] = 0;
                }
            for (int i = 0; i < n; i++) {
                for (int j = 0; j < 3; j++) cc[cidx[i]][j] += data[i][j];
                if (cnt[cidx[i]] == 0) comp[ncomp++] = cidx[i];
                cnt[cidx[i]]++;
            }
            for (int i = 0; i < ncomp; i++)
                for (int j = 0; j < 3; j++) cc[comp[i]][j] /= (float)cnt[comp[i]];
            for (int i = 0; i < ncomp; i++)
                for (int j = 0; j < 3; j++) cc[comp[i]][j] = floorf(cc[comp[i]][j] + 0.5f);
            float im[2][2] = {{0, 0}, {0, 0}}, rp[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
            for (int k = 0; k < n; k++) {
                im[0][0] += (float)((Mi_ - cidx[k]) * (Mi_ - cidx[k]));
                im[0][1] += (float)(cidx[k] * (Mi_ - cidx[k]));
                im[1][1] += (float)(cidx[k] * cidx[k]);
                for (int j = 0; j < 3; j++) {
                    rp[0][j] += (float)(Mi_ - cidx[k]) * cc[cidx[k]][j];
                    rp[1][j] += (float)cidx[k] * cc[cidx[k]][j];
                }
            }
            const float dd = im[0][0] * im[1][1] - im[0][1] * im[0][1];
            im[1][0] = im[0][0];
            im[0][0] = im[1][1] / dd;
            im[1][1] = im[1][0] / dd;
            im[1][0] = im[0][1] = -im[0][1] / dd;
            float epd[2][3][2];
            for (int j = 0; j < 3; j++) {
                const float e0 = (im[0][0] * rp[0][j] + im[0][1] * rp[1][j]) * (float)Mi_;
                const float e1 = (im[1][0] * rp[0][j] + im[1][1] * rp[1][j]) * (float)Mi_;
                const float ea[2] = {e0, e1};
                for (int i = 0; i < 2; i++) {
                    epd[i][j][0] = epd[i][j][1] = ea[i];
                    /* (1 << 8) - 1 - (int)epd, wrapping like the reference's int arithmetic */
                    const int lim = (int)(255u - (uint32_t)cvt_i32(epd[i][j][1]));
                    epd[i][j][1] += (float)(lim < 1 ? lim : 1);   /* use_par 0 */
                }
            }
            /* ce: per texel, cluster, channel squared distance of the corner */
            float ce[16][16][3];
            for (int i = 0; i < n; i++)
                for (int j = 0; j < ncl; j++)
                    for (int k = 0; k < 3; k++) {
                        const float r = ramp8(clog, cvt_i32(epd[0][k][0]), cvt_i32(epd[1][k][0]), j) - data[i][k];
                        ce[i][j][k] = r * r;
                    }
            float err_1 = FLT_MAX;
            int idx_1[16], s1 = 0, s = 0, ei0 = 0, ei1 = 0, j0 = 0;
            for (int p1 = 0; p1 < 64; p1++) {
                const int g = p1 & (-p1);
                for (int j = 0; j < 3; j++)
                    if (((g >> (2 * j)) & 0x3) != 0) {
                        j0 = j;
                        ei0 = ((s ^ g) >> (2 * j)) & 0x1;
                        ei1 = ((s ^ g) >> (2 * j + 1)) & 0x1;
                    }
                s = s ^ g;
                float err_0 = 0;
                int idx_0[16];
                for (int i = 0; i < n; i++) {
                    int ci = 0;
                    float cmin = FLT_MAX;
                    for (int j = 0; j < ncl; j++) {
                        const float r = ramp8(clog, cvt_i32(epd[0][j0][ei0]), cvt_i32(epd[1][j0][ei1]), j) - data[i][j0];
                        ce[i][j][j0] = r * r;
                        float t_ = 0.f;
                        for (int k = 0; k < 3; k++) t_ += ce[i][j][k];
                        if (t_ < cmin) {
                            cmin = t_;
                            ci = j;
                        }
                    }
                    idx_0[i] = ci;
                    err_0 += cmin;
                }
                if (err_0 < err_1) {
                    for (int i = 0; i < n; i++) idx_1[i] = idx_0[i];
                    err_1 = err_0;
                    s1 = s;
                }
            }
            int epo_1[2][4];
            for (int j = 0; j < 3; j++) {
                epo_1[0][j] = cvt_i32(epd[0][j][(s1 >> (2 * j)) & 0x1]);
                epo_1[1][j] = cvt_i32(epd[1][j][(s1 >> (2 * j + 1)) & 0x1]);
            }
            if (err_1 < err_2) {
                for (int i = 0; i < n; i++) idx_2[i] = idx_1[i];
                err_2 = err_1;
                for (int j = 0; j < 3; j++) {
                    epo_2[0][j] = epo_1[0][j];
                    epo_2[1][j] = epo_1[1][j];
                }
                p0 = p;
                q0 = q;
            }
        }
    (void)p0;
    (void)q0;
    if (err_2 < err_o) {
        for (int k = 0; k < n; k++) index_[k] = idx_2[k];
        for (int j = 0; j < 3; j++) {
            epo_code[0][j] = epo_2[0][j];
            epo_code[1][j] = epo_2[1][j];
        }
        err_o = err_2;
    }
    return err_o;
}

/* ------------------------------------------------------ FindBestPattern --- */

typedef struct {
    float din[16][4];
    int is_signed;
} bc6h_in;

typedef struct {
    float err;
    float fep[2][2][4];      /* fEndPoints after clampF16Max */
    int idx[2][16];          /* shape_indices (subset order) */
    int cnt[2];              /* entryCount */
} pattern_state;

/* palitizeEndPointsF (:707-758) + CalcShapeError (:783-836) */
static void palette(int region, float fep[2][2][4], float pal[2][16][3])
{
    if (region == 1) {
        for (int i = 0; i < 16; i++)
            for (int c = 0; c < 3; c++) pal[0][i][c] = lerp_pal(fep[0][0][c], fep[0][1][c], i, 15);
    } else {
        for (int r = 0; r < 2; r++)
            for (int i = 0; i < 8; i++)
                for (int c = 0; c < 3; c++) pal[r][i][c] = lerp_pal(fep[r][0][c], fep[r][1][c], i, 7);
    }
}

static float shape_error(const bc6h_in *in, int region, int shape, float pal[2][16][3])
{
    const int maxp = region == 1 ? 16 : 8;
    float total = 0.0f;
    for (int i = 0; i < 16; i++) {
        const int sub = region == 1 ? 0 : shape2_of(shape, i);
        float best = fabsf(in->din[i][0] - pal[sub][0][0]) + fabsf(in->din[i][1] - pal[sub][0][1]) +
                     fabsf(in->din[i][2] - pal[sub][0][2]);
        for (int j = 1; j < maxp && best > 0; j++) {
            const float e = fabsf(in->din[i][0] - pal[sub][j][0]) + fabsf(in->din[i][1] - pal[sub][j][1]) +
                            fabsf(in->din[i][2] - pal[sub][j][2]);
            if (e <= best)
                best = e;
            else
                break;
        }
        total += best;
    }
    return total;
}

/* clampF16Max (:510-529) on one end point value */
static float clamp_f16(float v, int is_signed)
{
    if (is_signed) {
        if (v < -F16MAX) return -F16MAX;
        if (v > F16MAX) return F16MAX;
    } else {
        if (v < 0.0) return 0;
        if (v > F16MAX) return F16MAX;
    }
    return v;
}

/* FindBestPattern (:904-1037) for pattern -1 (one region) or shape 0..31 */
static void find_pattern(const bc6h_in *in, int shape, pattern_state *st)
{
    const int two = shape >= 0;
    const int ns = two ? 2 : 1, ncl = two ? 8 : 16;
    float part[2][16][4];
    int cnt[2] = {0, 0};
    for (int i = 0; i < 16; i++) {   /* Partition :1069-1112 */
        const int sub = two ? shape2_of(shape, i) : 0;
        for (int j = 0; j < 3; j++) part[sub][cnt[sub]][j] = in->din[i][j];
        part[sub][cnt[sub]][3] = 0.0f;
        cnt[sub]++;
    }
    float outb[16][4];
    int idxb[2][2][16];
    float ep[2][2][4];
    memset(idxb, 0, sizeof(idxb));
    memset(ep, 0, sizeof(ep));
    float err0 = 0.0f, dir[4] = {0, 0, 0, 0};
    for (int s = 0; s < ns; s++) {
        err0 += opt_quant_f(part[s], cnt[s], ncl, idxb[0][s], outb, dir);
        /* GetEndPoints (:1116-1159): the quantised points of least / greatest
         * channel sum (first strictly smaller / greater) */
        float mn = HALF_MAX_F, mx = 0;
        int mini = 0, maxi = 0;
        for (int i = 0; i < cnt[s]; i++) {
            const float val = outb[i][0] + outb[i][1] + outb[i][2];
            if (val < mn) {
                mn = val;
                mini = i;
            }
            if (val > mx) {
                mx = val;
                maxi = i;
            }
        }
        for (int c = 0; c < 3; c++) {
            ep[s][0][c] = outb[mini][c];
            ep[s][1][c] = outb[maxi][c];
        }
    }
    float best = err0;
    int use_shaker = 0;
    int epo[2][2][4];
    memset(epo, 0, sizeof(epo));
    if (two) {   /* USE_SHAKERHD, quality 1.0 > 0.80 (:960-1025) */
        float err1 = 0.0f;
        for (int s = 0; s < ns; s++) {
            int tmp[16];
            for (int k = 0; k < cnt[s]; k++) tmp[k] = idxb[0][s][k];
            err1 += shaker_hd(part[s], cnt[s], tmp, epo[s]);
            for (int k = 0; k < cnt[s]; k++) idxb[1][s][k] = tmp[k];
        }
        if (best > err1) {
            best = err1;
            use_shaker = 1;
        }
    }
    (void)best;
    for (int s = 0; s < 2; s++)
        for (int e = 0; e < 2; e++)
            for (int c = 0; c < 3; c++) {
                const float v = use_shaker && s < ns ? (float)epo[s][e][c] : ep[s][e][c];
                st->fep[s][e][c] = clamp_f16(v, in->is_signed);
            }
    for (int s = 0; s < 2; s++)
        for (int k = 0; k < 16; k++) st->idx[s][k] = idxb[use_shaker][s][k];
    st->cnt[0] = cnt[0];
    st->cnt[1] = cnt[1];
    float pal[2][16][3];
    palette(ns, st->fep, pal);
    st->err = shape_error(in, ns, shape < 0 ? 0 : shape, pal);
}

/* ------------------------------------------------------- EncodePattern --- */

/* QuantizeToInt (amd_hdr_encode.cpp:83-115); (short) of the end point first */
static int quantize_to_int(short value, int prec, int is_signed)
{
    if (prec <= 1) return 0;
    int neg = 0;
    const int ivalue = value;
    if (is_signed) {
        if (value < 0) neg = 1;
        prec--;
    }
    int bias = (prec > 10 && prec != 16) ? ((1 << (prec - 11)) - 1) : 0;
    bias = (prec == 16) ? 15 : bias;
    /* the shift uses the original (signed) value */
    const int q = (int)(((long long)ivalue * (1LL << prec) + bias) / (F16MAX + 1));
    return neg ? -q : q;
}

static int is_overflow(int v, int nbit) { return !(v >= -(1 << (nbit - 1)) && v <= (1 << (nbit - 1)) - 1); }

/* TransformEndPoints (:598-660), two regions; returns 0 on overflow */
static int transform_ep(int mode, int ie[2][2][3], int oe[2][2][3], int *istransformed)
{
    const mode_part *mp = &kMP[mode];
    *istransformed = mp->transformed;
    for (int i = 0; i < 3; i++) {
        oe[0][0][i] = ie[0][0][i] & MASKN(mp->nbits);
        const int pm = MASKN(mp->prec[i]);
        if (mp->transformed) {
            oe[0][1][i] = ie[0][1][i] - ie[0][0][i];
            if (is_overflow(oe[0][1][i], mp->prec[i])) return 0;
            oe[0][1][i] &= pm;
            oe[1][0][i] = ie[1][0][i] - ie[0][0][i];
            if (is_overflow(oe[1][0][i], mp->prec[i])) return 0;
            oe[1][0][i] &= pm;
            oe[1][1][i] = ie[1][1][i] - ie[0][0][i];
            if (is_overflow(oe[1][1][i], mp->prec[i])) return 0;
            oe[1][1][i] &= pm;
        } else {
            oe[0][1][i] = ie[0][1][i] & pm;
            oe[1][0][i] = ie[1][0][i] & pm;
            oe[1][1][i] = ie[1][1][i] & pm;
        }
    }
    return 1;
}

/* endpts_fit (:493-507) with decompress_endpts (:458-490) */
static int endpoints_fit(int mode, int orig[2][2][3], int comp[2][2][3], int is_signed)
{
    const mode_part *mp = &kMP[mode];
    int un[2][2][3];
    for (int i = 0; i < 3; i++) {
        if (mp->transformed) {
            un[0][0][i] = is_signed ? sign_extend(comp[0][0][i], mp->index_prec) : comp[0][0][i];
            const int *src[3] = {&comp[0][1][i], &comp[1][0][i], &comp[1][1][i]};
            int *dst[3] = {&un[0][1][i], &un[1][0][i], &un[1][1][i]};
            for (int r = 0; r < 3; r++) {
                int t = sign_extend(*src[r], mp->prec[i]);
                t = (t + comp[0][0][i]) & MASKN(mp->nbits);
                *dst[r] = is_signed ? sign_extend(t, mp->nbits) : t;
            }
        } else {
            un[0][0][i] = is_signed ? sign_extend(comp[0][0][i], mp->nbits) : comp[0][0][i];
            un[0][1][i] = is_signed ? sign_extend(comp[0][1][i], mp->prec[i]) : comp[0][1][i];
            un[1][0][i] = is_signed ? sign_extend(comp[1][0][i], mp->prec[i]) : comp[1][0][i];
            un[1][1][i] = is_signed ? sign_extend(comp[1][1][i], mp->prec[i]) : comp[1][1][i];
        }
    }
    for (int j = 0; j < 2; ++j)
        for (int i = 0; i < 3; ++i)
            if (orig[j][0][i] != un[j][0][i] || orig[j][1][i] != un[j][1][i]) return 0;
    return 1;
}

/* Unquantize (:117-150, unsigned) + finish_unquantizeF16 (:1039-1049, unsigned) */
static float unq_f16(int comp, int bits)
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

/* decompress_endpoints2 (:1134-1252): the unsigned branches, `issigned` never set */
static void decode_ep2(int mode, int istr, int oe[2][2][3], float out[2][2][4])
{
    const mode_part *mp = &kMP[mode];
    for (int i = 0; i < 3; i++) {
        int o[2][2];
        o[0][0] = oe[0][0][i];
        if (istr) {
            o[0][1] = (sign_extend(oe[0][1][i], mp->prec[i]) + oe[0][0][i]) & MASKN(mp->nbits);
            o[1][0] = (sign_extend(oe[1][0][i], mp->prec[i]) + oe[0][0][i]) & MASKN(mp->nbits);
            o[1][1] = (sign_extend(oe[1][1][i], mp->prec[i]) + oe[0][0][i]) & MASKN(mp->nbits);
        } else {
            o[0][1] = oe[0][1][i];
            o[1][0] = oe[1][0][i];
            o[1][1] = oe[1][1][i];
        }
        for (int r = 0; r < 2; r++)
            for (int e = 0; e < 2; e++) out[r][e][i] = unq_f16(o[r][e], mp->nbits);
        out[0][0][3] = out[0][1][3] = out[1][0][3] = out[1][1][3] = 0;
    }
}

static void quantize_ep(float ep[2][2][4], int ie[2][2][3], int prec, int is_signed)
{
    for (int s = 0; s < 2; s++)
        for (int e = 0; e < 2; e++)
            for (int c = 0; c < 3; c++) ie[s][e][c] = quantize_to_int((short)cvt_i32(ep[s][e][c]), prec, is_signed);
}

/* SwapIndices (:555-581): anchors 0 and g_Region2FixUp[shape] */
static void swap_indices(int ie[2][2][3], int idx[2][16], const int cnt[2], int mode, int shape)
{
    const unsigned nidx = 1u << kMP[mode].index_prec, hi = nidx >> 1;
    for (int s = 0; s < 2; s++) {
        const int i = s ? anchor_pos(shape) : 0;
        if ((unsigned)idx[s][i] & hi) {
            for (int c = 0; c < 3; c++) {
                const int t = ie[s][0][c];
                ie[s][0][c] = ie[s][1][c];
                ie[s][1][c] = t;
            }
            for (int j = 0; j < cnt[s]; j++) idx[s][j] = (int)(nidx - 1u) - idx[s][j];
        }
    }
}

/* ReIndexShapef (:838-902), two regions: nearest palette entry, first strictly smaller */
static void reindex(const bc6h_in *in, int shape, float pal[2][16][3], int idx[2][16])
{
    int pos[2] = {0, 0};
    for (int i = 0; i < 16; i++) {
        const int sub = shape2_of(shape, i);
        float best = FLT_MAX;
        int bi = 0;
        for (int j = 0; j < 8; j++) {
            const float e = fabsf(in->din[i][0] - pal[sub][j][0]) + fabsf(in->din[i][1] - pal[sub][j][1]) +
                            fabsf(in->din[i][2] - pal[sub][j][2]);
            if (e < best) {
                best = e;
                bi = j;
            }
        }
        idx[sub][pos[sub]++] = bi;
    }
}

/* SaveDataBlock (:125-454), modes 1..10: (first bit, bits, field, shift) per
 * mode in the reference's order; fields 0..11 = rw gw bw rx gx bx ry gy by rz gz bz,
 * 12 = the mode value */
typedef struct {
    unsigned char start, bits, field, shift;
} bitfield;
enum { RW, GW, BW, RX, GX, BX, RY, GY, BY, RZ, GZ, BZ, MV };
static const bitfield kLayout[11][24] = {
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

/* BitHeader::setvalue (:88-100) */
static void set_bits(uint8_t b[16], int start, int bits, int value, int shift)
{
    int mask = 1 << shift;
    for (int k = 0; k < bits; k++, start++) {
        b[start / 8] = (uint8_t)(b[start / 8] & ~(1 << (start % 8)));
        b[start / 8] = (uint8_t)(b[start / 8] | (((value & mask) ? 1 : 0) << (start % 8)));
        mask <<= 1;
    }
}

static const uint8_t kRedBlock[16] = {0xc2, 0x7b, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
                                      0x00, 0xe0, 0x03, 0x00, 0x00, 0x00, 0x00, 0x00};

static void save_block(int mode, int shape, int oe[2][2][3], int idx[2][16], uint8_t out[16])
{
    int f[13];
    f[RW] = oe[0][0][0], f[GW] = oe[0][0][1], f[BW] = oe[0][0][2];
    f[RX] = oe[0][1][0], f[GX] = oe[0][1][1], f[BX] = oe[0][1][2];
    f[RY] = oe[1][0][0], f[GY] = oe[1][0][1], f[BY] = oe[1][0][2];
    f[RZ] = oe[1][1][0], f[GZ] = oe[1][1][1], f[BZ] = oe[1][1][2];
    f[MV] = kMP[mode].mode;
    memset(out, 0, 16);
    for (int k = 0; k < 24 && kLayout[mode][k].bits; k++) {
        const bitfield *bf = &kLayout[mode][k];
        set_bits(out, bf->start, bf->bits, f[bf->field], bf->shift);
    }
    /* indices in texel order (SaveCompressedBlockData :691-702), shape at 77 */
    set_bits(out, 77, 5, shape, 0);
    int pos[2] = {0, 0}, start = 82, nb = 2;
    const int anc = anchor_texel(shape);
    for (int i = 0; i < 16; i++) {
        const int sub = shape2_of(shape, i);
        const int v = idx[sub][pos[sub]++];
        if (i) {
            start += nb;
            nb = anc == i ? 2 : 3;
        }
        set_bits(out, start, nb, v, 0);
    }
}

/* EncodePattern (:1351-1488) for the two-region state; returns the error */
static float encode_pattern(const bc6h_in *in, int shape, const pattern_state *st, float error, uint8_t out[16])
{
    int best_fit = 0, numfits = 0;
    float best_err = FLT_MAX;
    int q_ep[11][2][2][3];
    int best_idx[11][2][16];
    for (int m = 1; m <= 10; ++m) {
        const mode_part *mp = &kMP[m];
        float ep[2][2][4];
        memcpy(ep, st->fep, sizeof(ep));
        memcpy(best_idx[m], st->idx, sizeof(best_idx[m]));
        int ie[2][2][3];
        quantize_ep(ep, ie, mp->nbits, in->is_signed);
        swap_indices(ie, best_idx[m], st->cnt, m, shape);
        int istr = 0;
        memset(q_ep[m], 0, sizeof(q_ep[m]));
        const int tfit = transform_ep(m, ie, q_ep[m], &istr);
        const int fits = tfit && endpoints_fit(m, ie, q_ep[m], in->is_signed);
        if (!fits) continue;
        numfits++;
        float unc[2][2][4];
        decode_ep2(m, istr, q_ep[m], unc);
        float pal[2][16][3];
        palette(2, unc, pal);
        if (!in->is_signed) reindex(in, shape, pal, best_idx[m]);
        const float e = shape_error(in, 2, shape, pal);
        if (e < best_err) {
            int tf = 1;
            if (!in->is_signed) {
                quantize_ep(unc, ie, mp->nbits, 0);
                swap_indices(ie, best_idx[m], st->cnt, m, shape);
                tf = transform_ep(m, ie, q_ep[m], &istr);
            }
            if (tf) {
                best_fit = m;
                best_err = e;
                error = e;
            }
        }
    }
    if (numfits > 0 && best_fit > 0)
        save_block(best_fit, shape, q_ep[best_fit], best_idx[best_fit], out);
    else
        memcpy(out, kRedBlock, 16);
    return error;
}

/* ------------------------------------------------------- CompressBlock --- */

/* texel conversion (:1539-1573) */
static void load_din(const float in[64], int is_signed, bc6h_in *b)
{
    b->is_signed = is_signed;
    for (int i = 0; i < 16; i++) {
        for (int c = 0; c < 3; c++) {
            const float v = in[i * 4 + c];
            if ((double)v < 0.00001) {
                const float a = fabsf(v / 1.0f);
                b->din[i][c] = is_signed ? (float)-(int)orc_float_to_half(a) : 0.0f;
            } else {
                b->din[i][c] = (float)orc_float_to_half(v / 1.0f);
            }
        }
        b->din[i][3] = 0.0f;
    }
}

float orc_bc6h_block(const float in[64], int is_signed, uint8_t out[16])
{
    bc6h_in b;
    load_din(in, is_signed, &b);
    pattern_state one, cur, best;
    find_pattern(&b, -1, &one);
    float best_err = one.err;
    int best_shape = -1;
    for (int shape = 0; shape < 32; ++shape) {
        find_pattern(&b, shape, &cur);
        if (cur.err < best_err) {
            best_err = cur.err;
            best_shape = shape;
            best = cur;
        }
    }
    /* the one-region pattern never beaten: the state left is shape 31's (:1621-1631) */
    const int shape = best_shape >= 0 ? best_shape : 31;
    const pattern_state *st = best_shape >= 0 ? &best : &cur;
    return encode_pattern(&b, shape, st, best_err, out);
}

/* test hook: FindBestPattern of one pattern (-1 = one region) */
float orc_bc6h_pattern(const float in[64], int is_signed, int shape, float fep[12], int idx[32], int cnt[2])
{
    bc6h_in b;
    load_din(in, is_signed, &b);
    pattern_state st;
    find_pattern(&b, shape, &st);
    for (int s = 0; s < 2; s++)
        for (int e = 0; e < 2; e++)
            for (int c = 0; c < 3; c++) fep[(s * 2 + e) * 3 + c] = st.fep[s][e][c];
    for (int s = 0; s < 2; s++)
        for (int k = 0; k < 16; k++) idx[s * 16 + k] = st.idx[s][k];
    cnt[0] = st.cnt[0];
    cnt[1] = st.cnt[1];
    return st.err;
}

int orc_bc6h_ev_p(void) { return ev_p(); }

/* ------------------------------------------------------- block batches --- */
#include <pthread.h>

typedef struct {
    const float *blocks;
    int n, is_signed;
    uint8_t *out;
    float *err;
    int next;
    pthread_mutex_t mu;
} bc6h_job;

static void *bc6h_worker(void *arg)
{
    bc6h_job *j = (bc6h_job *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        const int k = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (k >= j->n) break;
        const float e = orc_bc6h_block(j->blocks + (size_t)k * 64, j->is_signed, j->out + (size_t)k * 16);
        if (j->err) j->err[k] = e;
    }
    return NULL;
}

/* Image_CompressAMDBC6H's per-block call over n float RGBA blocks
 * (amd_bc6h_compressor.cpp:38-56), threads workers */
int orc_encode_bc6h_blocks(const float *blocks, int n, int is_signed, int threads, uint8_t *out, float *err)
{
    bc6h_job j;
    j.blocks = blocks;
    j.n = n;
    j.is_signed = is_signed;
    j.out = out;
    j.err = err;
    j.next = 0;
    pthread_mutex_init(&j.mu, NULL);
    if (threads <= 1) {
        bc6h_worker(&j);
    } else {
        pthread_t t[64];
        if (threads > 64) threads = 64;
        for (int i = 0; i < threads; ++i) pthread_create(&t[i], NULL, bc6h_worker, &j);
        for (int i = 0; i < threads; ++i) pthread_join(t[i], NULL);
    }
    pthread_mutex_destroy(&j.mu);
    return 0;
}

// gic_bc7.hip -- BC7 partition/mode search for gfx950 (MI355X).
//
// Algorithm: the reference's BC7 encoder at default quality
// (BC7BlockEncoder::CompressBlock, src/amd_bc7_body.cpp:1289-1465):
//   for every legal mode, for every partition: optQuantAnD_d per subset
//   (src/amd_bc7_3dquant_vpc.cpp:1874-2045) -> rank partitions (stable) ->
//   shake the best 8 with ep_shaker_d / ep_shaker_2_d (src/amd_shake.cpp) ->
//   pack; dual-index modes 4/5 over rotations x index selections.
// Arithmetic is IEEE f64 in the reference's order (-ffp-contract=off) so the
// output is bit-exact with the CPU restatement.  Shaker ramp values are
// evaluated with the exact integer identity
//   floor(e1 + (i/n)(e2-e1) + 0.5) = e1 + floor((2 i (e2-e1) + n) / 2n)
// (tests/test_oracle.py::test_shake_ramp_is_integer_lerp).
//
// Mapping (one chunk of blocks at a time, phases = kernels):
//   K0 prep    1 lane / block            texels x255, legal-mode mask
//   K1 quant   1 lane / (block, mode, partition)   273 tasks per block
//   K2 shake   1 lane / (block, mode, rank<8)      48 tasks per block
//   K3 dual    1 lane / (block, rotation, index selection) 12 tasks per block
//   K4 select  1 lane / block            mode choice + bit packing
// Each phase's lanes are independent; the reference's sequential "first
// strictly smaller" selections are reproduced by index-ordered reductions.
// The per-block workspace (~7 KB) lives in HBM between phases.

#include <vector>
#include <cstdlib>
#include <mutex>

#include "gic_common.h"
#include "bc7_tables.h"

namespace gic {
namespace bc7 {

enum { PAR_CART = 0, PAR_SAME = 1, PAR_BCC = 2 };
enum { ENC_NO_ALPHA = 0, ENC_COMBINED = 1, ENC_SEPARATE = 2 };

struct ModeInfo {
    int enc, part_bits, rot_bits, idxmode_bits, scalar_bits, vector_bits, pbit, subsets, ib0, ib1;
};

// bti[8], amd_bc7_body.cpp:84-94
__constant__ ModeInfo kModes[8] = {
    {ENC_NO_ALPHA, 4, 0, 0, 0, 12, 2, 3, 3, 0}, {ENC_NO_ALPHA, 6, 0, 0, 0, 18, 1, 2, 3, 0},
    {ENC_NO_ALPHA, 6, 0, 0, 0, 15, 0, 3, 2, 0}, {ENC_NO_ALPHA, 6, 0, 0, 0, 21, 2, 2, 2, 0},
    {ENC_SEPARATE, 0, 2, 1, 6, 15, 0, 1, 2, 3}, {ENC_SEPARATE, 0, 2, 0, 8, 21, 0, 1, 2, 2},
    {ENC_COMBINED, 0, 0, 0, 0, 28, 2, 1, 4, 0}, {ENC_COMBINED, 6, 0, 0, 0, 20, 2, 2, 2, 0},
};

__constant__ uint32_t dShape2[64];
__constant__ uint32_t dShape3[64];
__constant__ uint8_t dAnchor2[64];
__constant__ uint8_t dAnchor3a[64];
__constant__ uint8_t dAnchor3b[64];

// single-index task layout inside K1 / K2
constexpr int kQuantTasks = 273;   // m0:16, m1:64, m2:64, m3:64, m6:1, m7:64
constexpr int kShakeSlots = 6;     // modes 0,1,2,3,6,7
constexpr int kShakeRanks = 8;
constexpr uint32_t kSelectWaveBlocks = 4096;   // calls below this select with a wave per block
constexpr int kDualTasks = 12;     // mode 4: 4 rot x 2 sel, mode 5: 4 rot
// Distinct (subset mask, cluster count) problems among the subsets of modes
// 0-3's partitions (k_quant_sub): 150 with 8 clusters, 242 with 4, of 496.
constexpr int kUMax = 496;
__constant__ uint32_t dUProb[kUMax];      // mask | log2(clusters) << 16
__constant__ uint32_t dUMinPart[kUMax];   // byte m: lowest partition of mode m using it, 0xFF = none
__constant__ uint32_t dUMask[kUMax];      // distinct masks: u (8 clusters) | u (4 clusters) << 16, 0xFFFF = none
__constant__ uint16_t dTaskSub[208][3];   // task (modes 0-3) x subset -> problem, 0xFFFF = no subset
__constant__ int kSlotMode[6] = {0, 1, 2, 3, 6, 7};
__constant__ int kSlotBase[6] = {0, 16, 80, 144, 208, 209};

// single-point table of init_ramps (amd_shake.cpp:302-345), built on the host
struct SpEntry {
    int16_t p1, p2;
    uint32_t err;   // k*k, 0xffffffff = DBL_MAX
};
__device__ __forceinline__ int sp_index(int clog, int bits, int v, int o1, int o2, int i)
{
    return (((((clog - 2) * 4 + (bits - 5)) * 256 + v) * 2 + o1) * 2 + o2) * 16 + i;
}

struct BlockMeta {
    uint32_t valid;        // legal-mode mask after CompressBlock's filtering
    uint32_t pvalid;       // the same without the colour restriction (bounded-exit probes)
    uint32_t flags;        // bit0: unsupported (needs optQuantTrace_d), bit1: integral texels,
                           // bit2: error threshold met (staged low-quality pipeline) or
                           // final after the bounded-exit probe (k_bound)
    double max_range;
};

struct ShakeResult {
    double err[3];         // per-subset shake error (summed in subset order by k_select)
    uint64_t idx[3];       // per-subset texel indices, 4 bits per texel, texel order
    uint8_t ep[3][2][4];   // endpoint codes incl. parity bit (LSB) per subset
    uint32_t part;
    uint32_t pad;
};

struct DualResult {
    double err[2];         // colour, alpha (alpha divided by 3 when combined)
    uint64_t idx[2];       // 16 indices each, 4 bits per texel
    uint8_t ep[2][2][4];   // endpoint codes [half][endpoint][channel]
};

struct Workspace {
    float *tex;            // [n][64] inN * 255.0f
    BlockMeta *meta;       // [n]
    double *qerr;          // [n][273]
    uint64_t *qidx;        // [n][273]
    ShakeResult *shk;      // [n][6][8]
    DualResult *dual;      // [n][12]
    uint64_t *dqidx;       // [n][12][2] optQuantAnD_d indices of the dual-index candidates
    double *dqerr;         // [n][12][2] their optQuantAnD_d errors (quality <= 0.7 gating)
    double *best_err;      // [n] running best over the modes of earlier stages
    uint4 *best_blk;       // [n] its packed block
    double *uerr;          // [n][kUMax] optQuantAnD_d error of each distinct subset problem (modes 0-3)
    uint64_t *uidx;        // [n][kUMax] its indices, 4 bits per texel of the subset (texel order)
    uint8_t *prank;        // [n][6][8] partition of stable rank r of each single-index slot (k_rank)
    uint64_t *pqidx;       // [n][6][8] its optQuantAnD_d indices (k_rank), so a shake wave's loads are independent
    uint32_t *px;          // [n][16] texels packed R | G << 8 | B << 16 | A << 24 (integral blocks; k_prep)
    uint32_t *defer;       // [n][kDeferPer] shake problems the fast wave kernels handed to the slow ones
    uint32_t *defer_cnt;   // [4] their counts per kernel kind (zeroed per run_modes)
};

// Deferred shake problems (bc7_wave.inc FAST): list regions per kernel kind --
// k_shake_wave<8> (40 problems per block), <4> (56), <16> (1), k_dual_wave (24)
constexpr int kDeferPer = 121;
__host__ __device__ constexpr uint32_t defer_off(int kind) { return kind == 0 ? 0u : (kind == 1 ? 40u : (kind == 2 ? 96u : 97u)); }

__device__ __forceinline__ int expand_code(int bits, int v) { return (v << (8 - bits)) | (v >> (2 * bits - 8)); }

// ramp[clog][bits][p1][p2][i] of init_ramps (amd_shake.cpp:278-286), exactly
__device__ __forceinline__ int ramp_value(int clog, int bits, int p1, int p2, int i)
{
    const int e1 = expand_code(bits, p1), e2 = expand_code(bits, p2);
    const int n = (1 << clog) - 1;
    const int num = 2 * i * (e2 - e1) + n, den = 2 * n;
    int q = num / den;
    if (num < 0 && q * den != num) q--;
    return e1 + q;
}

__device__ __forceinline__ uint32_t shape_of(int subsets, int part, int texel)
{
    if (subsets == 1) return 0;
    const uint32_t m = subsets == 2 ? dShape2[part] : dShape3[part];
    return (m >> (2 * texel)) & 3u;
}

__device__ __forceinline__ int anchor_of(int subsets, int part, int s)
{
    if (s == 0) return 0;
    if (subsets == 2) return dAnchor2[part];
    return s == 1 ? dAnchor3a[part] : dAnchor3b[part];
}

// Iteration cap: optQuantAnD_d's requantisation loop
// `do ... while (!done && try_two--)` (amd_bc7_3dquant_vpc.cpp:1885,1986) never
// resets try_two, so once it has run negative the reference loops until the
// requantisation is stable -- forever on a cycling state.
//  * The register quantisers of the integral kernels (bc7_quant.inc) stop such a
//    loop g_iter_cap rounds past the counter's exhaustion, count the stop
//    (g_iter_hits) and mark the block (BlockMeta.flags bit 3 + the call's
//    re-run list, flag_capped).
//  * run_chunks then re-runs the marked blocks through the general kernels,
//    whose quantiser (opt_quant below) follows the reference's loop to its
//    fixed point.  The loop's state is the index vector alone, so a revisited
//    state proves the reference never returns: a Brent cycle check stops it
//    there and counts the block in g_nonterm (no output of the reference
//    exists for it).  kSafetyRounds bounds a pathological transient.
__device__ int g_iter_cap = 4096;
__device__ unsigned long long g_iter_hits = 0;
__device__ unsigned long long g_nonterm = 0;
constexpr int kSafetyRounds = 1 << 20;

// the reference's loop once try_two < 0: true = stop (cycle proven, or the
// safety bound); state = the index vector as 4-bit nibbles
struct CycleCheck {
    uint64_t saved = 0;
    int have = 0, pow = 1, lam = 0, rounds = 0;
    __device__ __forceinline__ bool stop(uint64_t st)
    {
        if (have && st == saved) {
            atomicAdd(&g_nonterm, 1ull);
            return true;
        }
        if (++rounds > kSafetyRounds) {
            atomicAdd(&g_iter_hits, 1ull);
            return true;
        }
        if (!have || ++lam == pow) {
            saved = st;
            have = 1;
            pow <<= 1;
            lam = 0;
        }
        return false;
    }
};

__device__ __forceinline__ int clog_of(int last)
{
    int c = 0, i = last + 1;
    while (i >>= 1) c++;
    return c;
}

// ep_find_floor, amd_shake.cpp:351-367
__device__ int ep_floor(double v, int bits, int use_par, int odd)
{
    int i1 = 0, i2 = 1 << (bits - use_par);
    odd = use_par ? odd : 0;
    while (i2 - i1 > 1) {
        const int j = (i1 + i2) / 2;
        if (v >= (double)expand_code(bits, (j << use_par) + odd))
            i1 = j;
        else
            i2 = j;
    }
    return (i1 << use_par) + odd;
}

// ------------------------------------------------------------ quantiser ---

// stable ascending sort of (value, index) pairs (glibc msort order)
__device__ void stable_sort(double *d, int *ix, int n)
{
    for (int i = 1; i < n; ++i) {
        const double t = d[i];
        const int ti = ix[i];
        int j = i - 1;
        while (j >= 0 && d[j] - t > 0) {
            d[j + 1] = d[j];
            ix[j + 1] = ix[j];
            --j;
        }
        d[j + 1] = t;
        ix[j + 1] = ti;
    }
}

// eigenVector_d, amd_bc7_3dquant_vpc.cpp:336-420 (p = 8 squarings, q = 3 rounds)
__device__ void principal_vector(double cov[4][4], double vec[4], int dim)
{
    double c[2][4][4];
    for (int i = 0; i < dim; ++i)
        for (int j = 0; j < dim; ++j) c[0][i][j] = cov[i][j];
    int l = 0;
    for (int n = 0; n < 3; ++n) {
        double md = 0;
        for (int i = 0; i < dim; ++i) md = c[l][i][i] > md ? c[l][i][i] : md;
        if (md <= 0) return;
        for (int i = 0; i < dim; ++i)
            for (int j = 0; j < dim; ++j) c[l][i][j] /= md;
        for (int m = 0; m < 8; ++m) {
            for (int i = 0; i < dim; ++i)
                for (int j = 0; j < dim; ++j) {
                    double t = 0;
                    for (int k = 0; k < dim; ++k) t += c[l][i][k] * c[l][k][j];
                    c[1 - l][i][j] = t;
                }
            l = 1 - l;
        }
    }
    double md = 0;
    int k = 0;
    for (int i = 0; i < dim; ++i) {
        k = c[l][i][i] > md ? i : k;
        md = c[l][i][i] > md ? c[l][i][i] : md;
    }
    double t = 0;
    for (int i = 0; i < dim; ++i) {
        t += c[l][k][i] * c[l][k][i];
        vec[i] = c[l][k][i];
    }
    t = sqrt(t);
    if (t <= 0) return;
    for (int i = 0; i < dim; ++i) vec[i] /= t;
}

// quant_AnD_Shell, amd_bc7_3dquant_vpc.cpp:1201-1286
__device__ void lattice_round(const double *v_, int k, int n, int *idx)
{
    double v[16], z[16], dd[16];
    int di[16];
    double m = v_[0], M = v_[0], dm = 0., r = 0;
    for (int i = 1; i < n; ++i) {
        m = m < v_[i] ? m : v_[i];
        M = M > v_[i] ? M : v_[i];
    }
    if (M == m) {
        for (int i = 0; i < n; ++i) idx[i] = 0;
        return;
    }
    const double s = (k - 1) / (M - m);
    for (int i = 0; i < n; ++i) {
        v[i] = v_[i] * s;
        idx[i] = (int)(z[i] = floor(v[i] + 0.5 - m * s));
        dd[i] = v[i] - z[i] - m * s;
        di[i] = i;
        dm += dd[i];
        r += dd[i] * dd[i];
    }
    if (n * r - dm * dm >= (double)(n - 1) / 4 / 2) {
        dm /= (double)n;
        for (int i = 0; i < n; ++i) dd[i] -= dm;
        stable_sort(dd, di, n);
        for (int i = 0; i < n; ++i) dd[i] -= (2. * (double)i + 1 - (double)n) / 2. / (double)n;
        double mm = 0., l = 0.;
        int j = -1;
        for (int i = 0; i < n; ++i) {
            l += dd[i];
            if (l < mm) {
                mm = l;
                j = i;
            }
        }
        j = (j + 1) % n;
        for (int i = j; i < n; ++i) idx[di[i]]++;
    }
    int mi = idx[0];
    for (int i = 1; i < n; ++i) mi = mi < idx[i] ? mi : idx[i];
    for (int i = 0; i < n; ++i) idx[i] -= mi;
}

__device__ __forceinline__ void project(const double cen[][4], int n, const double *v, double *out, int dim)
{
    for (int k = 0; k < n; ++k) {
        out[k] = 0;
        for (int i = 0; i < dim; ++i) out[k] += cen[k][i] * v[i];
    }
}

// optQuantAnD_d, amd_bc7_3dquant_vpc.cpp:1874-2045 (n <= 16 here)
__device__ double opt_quant(const double data[][4], int n, int ncl, int *index, int dim)
{
    int snap[16], order[16];
    double cen[16][4], mean[4], cov[4][4], prj[16], dir[4] = {0, 0, 0, 0};
    double s, t;
    int try_two = 50;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < dim; ++j) cen[i][j] = data[i][j];
    for (int i = 0; i < dim; ++i) {
        mean[i] = 0;
        for (int k = 0; k < n; ++k) mean[i] += cen[k][i];
    }
    if (n) {
        for (int i = 0; i < dim; ++i) {
            mean[i] /= (double)n;
            for (int k = 0; k < n; ++k) cen[k][i] -= mean[i];
        }
    }
    for (int i = 0; i < dim; ++i)
        for (int j = 0; j <= i; ++j) {
            cov[i][j] = 0;
            for (int k = 0; k < n; ++k) cov[i][j] += cen[k][i] * cen[k][j];
        }
    for (int i = 0; i < dim; ++i)
        for (int j = i + 1; j < dim; ++j) cov[i][j] = cov[j][i];
    t = 0;
    for (int j = 0; j < dim; ++j) t += cov[j][j];
    if (t < (1. / 256.) || n == 0) {
        // every point quantises to the mean: error = sum |x - mean|^2 ... but
        // the reference returns 0 here (amd_bc7_3dquant_vpc.cpp:1914-1921)
        for (int i = 0; i < n; ++i) index[i] = 0;
        return 0.;
    }
    principal_vector(cov, dir, dim);
    project(cen, n, dir, prj, dim);
    for (int it = 0; it < 200; ++it) {
        if (it) {
            int done;
            CycleCheck cyc;   // per requantisation loop: a state seen in an earlier loop proves nothing
            do {
                double q = 0;
                s = t = 0;
                for (int k = 0; k < n; ++k) {
                    s += index[k];
                    t += index[k] * index[k];
                }
                for (int j = 0; j < dim; ++j) {
                    dir[j] = 0;
                    for (int k = 0; k < n; ++k) dir[j] += cen[k][j] * index[k];
                    q += dir[j] * dir[j];
                }
                s /= (double)n;
                t = t - s * s * (double)n;
                t = (t == 0 ? 0. : 1 / t);
                q = sqrt(q);
                t *= q;
                if (q != 0)
                    for (int j = 0; j < dim; ++j) dir[j] /= q;
                project(cen, n, dir, prj, dim);
                double sd[16];
                for (int j = 0; j < n; ++j) {
                    sd[j] = prj[j];
                    order[j] = j;
                }
                stable_sort(sd, order, n);
                int nidx[16], k = 0;
                for (int j = 0; j < n; ++j) {
                    while (prj[order[j]] > (k + 0.5 - s) * t && k < ncl - 1) k++;
                    nidx[order[j]] = k;
                }
                done = 1;
                uint64_t st = 0;
                for (int j = 0; j < n; ++j) {
                    done = (done && (nidx[j] == index[j]));
                    index[j] = nidx[j];
                    st |= (uint64_t)(nidx[j] & 15) << (4 * j);
                }
                // the reference's counter is never reset; past zero the loop
                // runs until the requantisation is stable (or, on a cycle, forever)
                if (!done && try_two < 0 && cyc.stop(st)) break;
            } while (!done && try_two--);
            if (it == 1) {
                for (int j = 0; j < n; ++j) snap[j] = index[j];
            } else {
                done = 1;
                for (int j = 0; j < n; ++j) done = (done && (snap[j] == index[j]));
                if (done) break;
            }
        }
        lattice_round(prj, ncl, n, index);
    }
    double q = 0;
    s = t = 0;
    for (int k = 0; k < n; ++k) {
        s += index[k];
        t += index[k] * index[k];
    }
    for (int j = 0; j < dim; ++j) {
        dir[j] = 0;
        for (int k = 0; k < n; ++k) dir[j] += cen[k][j] * index[k];
        q += dir[j] * dir[j];
    }
    s /= (double)n;
    t = t - s * s * (double)n;
    t = (t == 0 ? 0. : 1 / t);
    double err = 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < dim; ++j) {
            const double o = mean[j] + dir[j] * t * (index[i] - s);
            err += (data[i][j] - o) * (data[i][j] - o);
        }
    return err;
}

#define GIC_QUANT_CAP g_iter_cap
#define GIC_QUANT_CAP_HIT atomicAdd(&g_iter_hits, 1ull)
#include "bc7_quant.inc"

// ------------------------------------ exhaustive quantiser (performance < 1) ---
// optQuantTrace_d (amd_bc7_3dquant_vpc.cpp:1425-1554) with quantTrace_d
// (:1067-1199) walking the traceBuilder tables (:1557-1712), which the host
// builds once per device (build_trace below).  Step i of table (nc, ne) holds
// kc = k | code << 5 (k = 2 * entry + 1 if the entry leaves its cluster
// downwards, the sign of its contribution) and d = 1 / (q2 - q^2 / ne).  The
// reference's encoder calls it instead of optQuantAnD_d for blocks whose range
// exceeds 255 * performance, single-index modes with at most 8 clusters
// (amd_bc7_body.cpp:606-633) and both halves of the dual-index candidates
// (:1103-1154).  One lane per problem: the walk's double sums run in the
// reference's order.
struct TraceTab {
    const uint32_t *kc;
    const double *d;
};
__constant__ uint32_t dTraceOff[8][16];
__constant__ uint32_t dTraceCnt[8][16];

__device__ void quant_trace(const double ord[][4], int ne, int nc, int *index, int dim, const TraceTab &tt)
{
    const uint32_t off = dTraceOff[nc - 1][ne - 1], cnt = dTraceCnt[nc - 1][ne - 1];
    double acc[4] = {0., 0., 0., 0.}, best = 0.;
    int k = -1;
    for (uint32_t i = 0; i < cnt; ++i) {
        const uint32_t kc = tt.kc[off + i];
        const int e = (int)((kc & 31u) >> 1);
        const bool neg = kc & 1u;
        double c = 0.;
        for (int j = 0; j < dim; ++j) {
            acc[j] += neg ? -ord[e][j] : ord[e][j];
            c = j ? c + acc[j] * acc[j] : acc[j] * acc[j];
        }
        c = c * tt.d[off + i];
        if (c > best) {
            best = c;
            k = (int)i;
        }
    }
    if (k < 0) {
        for (int i = 0; i < ne; ++i) index[i] = 0;
        return;
    }
    uint32_t bits = tt.kc[off + (uint32_t)k] >> 5;
    int cl = 0;
    for (int i = 0; i < ne; ++i) {
        while (!(bits & 1u)) {
            ++cl;
            bits >>= 1;
        }
        index[i] = cl;
        bits >>= 1;
    }
}

__device__ double opt_quant_trace(const double data[][4], int n, int ncl, int *index_, int dim, const TraceTab &tt)
{
    int index[16], order[16];
    double cen[16][4], ord[16][4], mean[4], cov[4][4], prj[16], dir[4] = {0, 0, 0, 0};
    double s, t = 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < dim; ++j) cen[i][j] = data[i][j];
    for (int i = 0; i < dim; ++i) {   // centerInPlace_d
        mean[i] = 0;
        for (int k = 0; k < n; ++k) mean[i] += cen[k][i];
    }
    if (n)
        for (int i = 0; i < dim; ++i) {
            mean[i] /= (double)n;
            for (int k = 0; k < n; ++k) cen[k][i] -= mean[i];
        }
    for (int i = 0; i < dim; ++i)   // covariance_d
        for (int j = 0; j <= i; ++j) {
            cov[i][j] = 0;
            for (int k = 0; k < n; ++k) cov[i][j] += cen[k][i] * cen[k][j];
        }
    for (int i = 0; i < dim; ++i)
        for (int j = i + 1; j < dim; ++j) cov[i][j] = cov[j][i];
    for (int j = 0; j < dim; ++j) t += cov[j][j];
    if (t < 0.000001 || n == 0) {   // EPSILON
        for (int i = 0; i < n; ++i) index_[i] = 0;
        return 0.;   // every entry at the mean: no error
    }
    principal_vector(cov, dir, dim);
    project(cen, n, dir, prj, dim);
    for (int it = 0; it < 20; ++it) {   // MAX_TRY
        if (it) {   // re-project on the least-squares direction; stop once the order holds
            t = 0;
            for (int j = 0; j < dim; ++j) {
                dir[j] = 0;
                for (int k = 0; k < n; ++k) dir[j] += ord[k][j] * index[k];
                t += dir[j] * dir[j];
            }
            t = sqrt(t) * 0.000001;
            project(cen, n, dir, prj, dim);
            int j = 1;
            while (j < n && !(prj[order[j]] < prj[order[j - 1]] - t)) ++j;
            if (j >= n) break;
        }
        double sd[16];
        for (int k = 0; k < n; ++k) sd[k] = prj[k], order[k] = k;
        stable_sort(sd, order, n);   // sortProjection
        for (int k = 0; k < n; ++k)
            for (int j = 0; j < dim; ++j) ord[k][j] = cen[order[k]][j];
        quant_trace(ord, n, ncl, index, dim, tt);
    }
    s = t = 0;
    for (int k = 0; k < n; ++k) {
        s += index[k];
        t += index[k] * index[k];
    }
    for (int j = 0; j < dim; ++j) {
        dir[j] = 0;
        for (int k = 0; k < n; ++k) dir[j] += ord[k][j] * index[k];
    }
    s /= (double)n;
    t = t - s * s * (double)n;
    t = (t == 0 ? 0. : 1 / t);
    for (int i = 0; i < n; ++i) index_[order[i]] = index[i];
    double err = 0;   // totalError_d over the entries in their own order
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < dim; ++j) {
            const double o = mean[j] + dir[j] * t * (index_[i] - s);
            err += (data[i][j] - o) * (data[i][j] - o);
        }
    return err;
}

// -------------------------------------------------------------- shakers ---

__device__ void collapse(int *idx, int n)
{
    if (!n) return;
    int mi = idx[0], Mi = idx[0], D = 1;
    for (int k = 1; k < n; ++k) {
        mi = mi < idx[k] ? mi : idx[k];
        Mi = Mi > idx[k] ? Mi : idx[k];
    }
    for (int d = 2; d <= Mi - mi; ++d) {
        int k;
        for (k = 0; k < n; ++k)
            if ((idx[k] - mi) % d != 0) break;
        if (k >= n) D = d;
    }
    for (int k = 0; k < n; ++k) idx[k] = (idx[k] - mi) / D;
}

__device__ __forceinline__ int max_index(const int *a, int n)
{
    int m = a[0];
    for (int i = 0; i < n; ++i) m = m > a[i] ? m : a[i];
    return m;
}

__device__ int all_same(const double d[][4], int n, int dim)
{
    int same = 1;
    for (int i = 1; i < n; ++i)
        for (int j = 0; j < dim; ++j) same = same && (d[0][j] == d[i][j]);
    return same;
}

__device__ void mean_of(const double d[][4], double mean[4], int n, int dim)
{
    for (int j = 0; j < dim; ++j) mean[j] = 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < dim; ++j) mean[j] += d[i][j];
    for (int j = 0; j < dim; ++j) mean[j] /= (double)n;
}

__constant__ int kParCount[3] = {1, 2, 4};
__constant__ int kParVec[3][4][2] = {{{0, 0}}, {{0, 0}, {1, 1}}, {{0, 0}, {0, 1}, {1, 0}, {1, 1}}};

__device__ __forceinline__ double sp_err(const SpEntry *sp, int c, int b, int v, int o1, int o2, int i)
{
    const uint32_t e = sp[sp_index(c + 2, b + 5, v, o1, o2, i)].err;
    return e == 0xffffffffu ? 1.7976931348623157e308 : (double)e;
}

// quant_single_point_d, amd_shake.cpp:546-701: best (cluster, endpoint pair)
// for one point; returns err1 (per point) and the cluster index in idx_out.
__device__ double single_point_core(const SpEntry *sp, const double point[4], int &idx_out, int epo1[2][4],
                                    int last, const int *bits, int type, int dim)
{
    double err0 = 1.7976931348623157e308, err1 = 1.7976931348623157e308;
    int idx = 0, idx1 = 0, epo0[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    const int use_par = (type != 0);
    const int clog = clog_of(last), c = clog - 2;
    for (int pn = 0; pn < kParCount[type]; ++pn) {
        int lo1[4], hi1[4], lo2[4], hi2[4];
        for (int j = 0; j < dim; ++j) {
            lo1[j] = lo2[j] = 0;
            hi1[j] = hi2[j] = 2;
            if (use_par) {
                if (kParVec[type][pn][0]) lo1[j] = 1; else hi1[j] = 1;
                if (kParVec[type][pn][1]) lo2[j] = 1; else hi2[j] = 1;
            }
        }
        for (int i = 0; i < (1 << clog); ++i) {
            double t = 0;
            int t1o[4] = {0, 0, 0, 0}, t2o[4] = {0, 0, 0, 0}, dr0[4] = {0, 0, 0, 0};
            for (int j = 0; j < dim; ++j) {
                double tbest = 1.7976931348623157e308;
                const int b = bits[j] - 5;
                for (int t1 = lo1[j]; t1 < hi1[j]; ++t1)
                    for (int t2 = lo2[j]; t2 < hi2[j]; ++t2) {
                        int tf = (int)floor(point[j]);
                        int tc = (int)ceil(point[j]);
                        tf = (tf < 0) ? 0 : tf;
                        tc = (tc > 255) ? 255 : tc;
                        const double ef = sp_err(sp, c, b, tf, t1, t2, i), ec = sp_err(sp, c, b, tc, t1, t2, i);
                        int dr;
                        if (ef > ec)
                            dr = tc;
                        else if (ef < ec)
                            dr = tf;
                        else
                            dr = (int)floor(point[j] + 0.5);
                        const double e = sp_err(sp, c, b, dr, t1, t2, i);
                        const double tr = e + 2 * sqrt(e) * fabs((double)dr - point[j]) +
                                          (dr - point[j]) * (dr - point[j]);
                        if (tr < tbest) {
                            tbest = tr;
                            t1o[j] = t1;
                            t2o[j] = t2;
                            dr0[j] = dr;
                        }
                    }
                t += tbest;
            }
            if (t < err0) {
                idx = i;
                for (int j = 0; j < dim; ++j) {
                    const SpEntry &e = sp[sp_index(clog, bits[j], dr0[j], t1o[j], t2o[j], i)];
                    epo0[0][j] = e.p1;
                    epo0[1][j] = e.p2;
                }
                err0 = t;
            }
            if (err0 == 0) break;
        }
        if (err0 < err1) {
            idx1 = idx;
            for (int j = 0; j < dim; ++j) {
                epo1[0][j] = epo0[0][j];
                epo1[1][j] = epo0[1][j];
            }
            err1 = err0;
        }
        if (err1 == 0) break;
    }
    idx_out = idx1;
    return err1;
}

// Returns err1 * n, or, when `data` is given (not all-same path), the
// totalError_d of the reconstruction against it.
__device__ double single_point(const SpEntry *sp, const double point[4], int n, int *index, int epo1[2][4],
                               int last, const int *bits, int type, int dim, const double (*data)[4])
{
    int idx1;
    const double err1 = single_point_core(sp, point, idx1, epo1, last, bits, type, dim);
    const int clog = clog_of(last);
    for (int i = 0; i < n; ++i) index[i] = idx1;
    if (!data) return err1 * n;
    double t = 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < dim; ++j) {
            const double o = (double)ramp_value(clog, bits[j], epo1[0][j], epo1[1][j], idx1);
            t += (data[i][j] - o) * (data[i][j] - o);
        }
    return t;
}

// least squares endpoints for an expanded index (amd_shake.cpp:837-886)
__device__ void ls_endpoints(const double data[][4], const int *cidx, int n, int last, int dim, double epa[2][4])
{
    double im[2][2] = {{0, 0}, {0, 0}}, rp[2][4], cc[16][4];
    int cnt[16], comp[16], ncl = 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < dim; ++j) {
            cc[cidx[i]][j] = 0;
            cnt[cidx[i]] = 0;
        }
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j < dim; ++j) cc[cidx[i]][j] += data[i][j];
        if (cnt[cidx[i]] == 0) comp[ncl++] = cidx[i];
        cnt[cidx[i]]++;
    }
    for (int i = 0; i < ncl; ++i)
        for (int j = 0; j < dim; ++j) cc[comp[i]][j] /= (double)cnt[comp[i]];
    for (int i = 0; i < ncl; ++i)
        for (int j = 0; j < dim; ++j) cc[comp[i]][j] = floor(cc[comp[i]][j] + 0.5);
    for (int j = 0; j < dim; ++j) rp[0][j] = rp[1][j] = 0;
    for (int k = 0; k < n; ++k) {
        im[0][0] += (last - cidx[k]) * (last - cidx[k]);
        im[0][1] += cidx[k] * (last - cidx[k]);
        im[1][1] += cidx[k] * cidx[k];
        for (int j = 0; j < dim; ++j) {
            rp[0][j] += (last - cidx[k]) * cc[cidx[k]][j];
            rp[1][j] += cidx[k] * cc[cidx[k]][j];
        }
    }
    const double dd = im[0][0] * im[1][1] - im[0][1] * im[0][1];
    im[1][0] = im[0][0];
    im[0][0] = im[1][1] / dd;
    im[1][1] = im[1][0] / dd;
    im[1][0] = im[0][1] = -im[0][1] / dd;
    for (int j = 0; j < dim; ++j) {
        epa[0][j] = (im[0][0] * rp[0][j] + im[0][1] * rp[1][j]) * last;
        epa[1][j] = (im[1][0] * rp[0][j] + im[1][1] * rp[1][j]) * last;
    }
}

template <typename T> struct Limits;
template <> struct Limits<int> { __device__ static int max() { return 0x7fffffff; } };
template <> struct Limits<double> { __device__ static double max() { return 1.7976931348623157e308; } };

// ep_shaker_2_d, amd_shake.cpp:703-1053.  index_ and epo_code updated in place.
// All window / requantisation errors are sums of squared differences of
// integers and are computed exactly in int32.
template <typename T>
__device__ double shake_window(const SpEntry *sp, const double data[][4], const T *idata, int n, int *index_,
                               int epo_code[2][4], int size, int last, int bits, int dim)
{
    const int type = bits % (2 * dim);
    const int use_par = (type != 0);
    int mb[4];
    for (int j = 0; j < dim; ++j) mb[j] = (bits + 2 * dim - 1) / (2 * dim);
    const int clog = clog_of(last), nc = 1 << clog;
    double mean[4], err_o = 1.7976931348623157e308;
    int index[16], epo0[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    int max_try = 8, done;
    for (int k = 0; k < n; ++k) index[k] = index_[k];
    const int alls = all_same(data, n, dim);
    mean_of(data, mean, n, dim);
    do {
        collapse(index, n);
        const int Mi = max_index(index, n);
        int p0 = -1, q0 = -1;
        double err0 = 1.7976931348623157e308;
        if (Mi == 0) {
            int tidx[16];
            const double t = alls ? single_point(sp, data[0], n, tidx, epo0, last, mb, type, dim, nullptr)
                                  : single_point(sp, mean, n, tidx, epo0, last, mb, type, dim, data);
            if (t < err_o) {
                for (int k = 0; k < n; ++k) index_[k] = tidx[k];
                for (int j = 0; j < dim; ++j) {
                    epo_code[0][j] = epo0[0][j];
                    epo_code[1][j] = epo0[1][j];
                }
                err_o = t;
            }
            return err_o;
        }
        for (int q = 1; q * Mi <= last; ++q)
            for (int p = 0; p <= last - q * Mi; ++p) {
                int cidx[16];
                double epa[2][4];
                for (int k = 0; k < n; ++k) cidx[k] = index[k] * q + p;
                ls_endpoints(data, cidx, n, last, dim, epa);
                T ed[2][2][4];
                int best2[2][2][2][4];
                for (int j = 0; j < dim; ++j) {
                    const int rr = use_par ? 2 : 1;
                    for (int a = 0; a < rr; ++a)
                        for (int b = 0; b < rr; ++b) {
                            int lo[2], hi[2];
                            const int pp[2] = {a, b};
                            for (int i = 0; i < 2; ++i) {
                                const int f = ep_floor(epa[i][j], mb[j], use_par, pp[i]);
                                lo[i] = hi[i] = f;
                                lo[i] -= ((f < (size >> 1) - 1) ? f : (size >> 1) - 1) & (~use_par);
                                hi[i] += (((1 << mb[j]) - 1 - f < (size >> 1)) ? (1 << mb[j]) - 1 - f : (size >> 1)) &
                                         (~use_par);
                            }
                            const int step = 1 << use_par;
                            T best = Limits<T>::max();
                            for (int p1 = lo[0]; p1 <= hi[0]; p1 += step)
                                for (int p2 = lo[1]; p2 <= hi[1]; p2 += step) {
                                    T t = 0;
                                    for (int m = n; m > 0; --m) {   // reverse texel order (amd_shake.cpp:934-938)
                                        const T d = (T)ramp_value(clog, mb[j], p1, p2, cidx[m - 1]) - idata[(m - 1) * 4 + j];
                                        t += d * d;
                                    }
                                    if (t < best) {
                                        best = t;
                                        best2[a][b][0][j] = p1;
                                        best2[a][b][1][j] = p2;
                                    }
                                }
                            ed[a][b][j] = best;
                        }
                }
                T err1 = Limits<T>::max();
                int epo1[2][4];
                for (int pn = 0; pn < kParCount[type]; ++pn) {
                    const int v0 = kParVec[type][pn][0], v1 = kParVec[type][pn][1];
                    T e2 = 0;
                    for (int j = 0; j < dim; ++j) e2 += ed[v0][v1][j];
                    if (e2 < err1) {
                        err1 = e2;
                        for (int j = 0; j < dim; ++j) {
                            epo1[0][j] = best2[v0][v1][0][j];
                            epo1[1][j] = best2[v0][v1][1][j];
                        }
                    }
                }
                if ((double)err1 <= err0) {   // Q7: last minimum wins (amd_shake.cpp:970)
                    err0 = (double)err1;
                    p0 = p;
                    q0 = q;
                    for (int j = 0; j < dim; ++j) {
                        epo0[0][j] = epo1[0][j];
                        epo0[1][j] = epo1[1][j];
                    }
                }
            }
        // requantise (amd_shake.cpp:980-1018)
        int idg[16];
        T err_r = 0;
        for (int i = 0; i < n; ++i) {
            T cmin = Limits<T>::max();
            int ci = 0;
            for (int c = 0; c < nc; ++c) {
                T t = 0;
                for (int k = 0; k < dim; ++k) {
                    const T d = (T)ramp_value(clog, mb[k], epo0[0][k], epo0[1][k], c) - idata[i * 4 + k];
                    t += d * d;
                }
                if (t < cmin) {
                    cmin = t;
                    ci = c;
                }
            }
            idg[i] = ci;
            err_r += cmin;
        }
        int change = 0;
        for (int k = 0; k < n; ++k) change = change || (index[k] * q0 + p0 != idg[k]);
        const int better = (double)err_r < err_o;
        if (better) {
            for (int k = 0; k < n; ++k) index_[k] = index[k] = idg[k];
            for (int j = 0; j < dim; ++j) {
                epo_code[0][j] = epo0[0][j];
                epo_code[1][j] = epo0[1][j];
            }
            err_o = (double)err_r;
        }
        done = !(change && better);
    } while (!done && max_try--);
    return err_o;
}

// ep_shaker_d, amd_shake.cpp:1058-1404 (dimension 3).  Corner errors are
// exact integers; the 64-corner Gray-code walk is evaluated corner by corner.
template <typename T>
__device__ double shake_corners(const SpEntry *sp, const double data[][4], const T *idata, int n, int *index_,
                                int epo_code[2][4], int last, const int *bits, int type)
{
    const int dim = 3;
    const int use_par = (type == PAR_BCC || type == PAR_SAME);
    const int bcc = (type == PAR_BCC);
    const int clog = clog_of(last), nc = 1 << clog;
    double mean[4], err_o = 1.7976931348623157e308;
    int index[16], max_try = 1, done;
    for (int k = 0; k < n; ++k) index[k] = index_[k];
    const int alls = all_same(data, n, dim);
    mean_of(data, mean, n, dim);
    do {
        collapse(index, n);
        const int Mi = max_index(index, n);
        int p0 = -1, q0 = -1, idx2[16], epo2[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
        T err2 = Limits<T>::max();
        if (Mi == 0) {
            int epo0[2][4], tidx[16];
            const double t = alls ? single_point(sp, data[0], n, tidx, epo0, last, bits, type, dim, nullptr)
                                  : single_point(sp, mean, n, tidx, epo0, last, bits, type, dim, data);
            if (t < err_o) {
                for (int k = 0; k < n; ++k) index_[k] = tidx[k];
                for (int j = 0; j < dim; ++j) {
                    epo_code[0][j] = epo0[0][j];
                    epo_code[1][j] = epo0[1][j];
                }
                err_o = t;
            }
            return err_o;
        }
        for (int k = 0; k < n; ++k) idx2[k] = 0;
        for (int q = 1; q * Mi <= last; ++q)
            for (int p = 0; p <= last - q * Mi; ++p) {
                int cidx[16], idx1[16], epo1[2][4], s1 = 0;
                T err1 = Limits<T>::max();
                double epa[2][4];
                for (int k = 0; k < n; ++k) cidx[k] = index[k] * q + p;
                ls_endpoints(data, cidx, n, last, dim, epa);
                for (int odd = 0; odd <= use_par; ++odd)
                    for (int flip = 0; flip <= bcc; ++flip) {
                        int epi[2][3][2];
                        for (int j = 0; j < dim; ++j)
                            for (int i = 0; i < 2; ++i) {
                                const int f = ep_floor(epa[i][j], bits[j], use_par, (odd ^ (flip & i)) & 1);
                                epi[i][j][0] = epi[i][j][1] = f;
                                epi[i][j][1] += (((1 << bits[j]) - 1 - f < (1 << use_par)) ? (1 << bits[j]) - 1 - f
                                                                                            : (1 << use_par)) &
                                                (~use_par);
                            }
                        int s = 0;
                        for (int p1 = 0; p1 < 64; ++p1) {
                            s ^= p1 & (-p1);
                            int r[3][16];
                            for (int j = 0; j < dim; ++j) {
                                const int a = epi[0][j][(s >> (2 * j)) & 1], b = epi[1][j][(s >> (2 * j + 1)) & 1];
                                for (int c = 0; c < nc; ++c) r[j][c] = ramp_value(clog, bits[j], a, b, c);
                            }
                            T err0 = 0;
                            int idx0[16];
                            for (int i = 0; i < n; ++i) {
                                int ci = 0;
                                T cmin = Limits<T>::max();
                                for (int c = 0; c < nc; ++c) {
                                    const T d0 = (T)r[0][c] - idata[i * 4 + 0];
                                    const T d1 = (T)r[1][c] - idata[i * 4 + 1];
                                    const T d2 = (T)r[2][c] - idata[i * 4 + 2];
                                    const T t = d0 * d0 + d1 * d1 + d2 * d2;
                                    if (t < cmin) {
                                        cmin = t;
                                        ci = c;
                                    }
                                }
                                idx0[i] = ci;
                                err0 += cmin;
                            }
                            if (err0 < err1) {
                                for (int i = 0; i < n; ++i) idx1[i] = idx0[i];
                                err1 = err0;
                                s1 = s;
                            }
                        }
                        // Q6: endpoints rebuilt from the global s1 with this pass's ranges
                        for (int j = 0; j < dim; ++j) {
                            epo1[0][j] = epi[0][j][(s1 >> (2 * j)) & 1];
                            epo1[1][j] = epi[1][j][(s1 >> (2 * j + 1)) & 1];
                        }
                    }
                if (err1 < err2) {
                    for (int i = 0; i < n; ++i) idx2[i] = idx1[i];
                    err2 = err1;
                    for (int j = 0; j < dim; ++j) {
                        epo2[0][j] = epo1[0][j];
                        epo2[1][j] = epo1[1][j];
                    }
                    p0 = p;
                    q0 = q;
                }
            }
        int change = 0;
        for (int k = 0; k < n; ++k) change = change || (index[k] * q0 + p0 != idx2[k]);
        const int better = (double)err2 < err_o;
        if (better) {
            for (int k = 0; k < n; ++k) index_[k] = index[k] = idx2[k];
            for (int j = 0; j < dim; ++j) {
                epo_code[0][j] = epo2[0][j];
                epo_code[1][j] = epo2[1][j];
            }
            err_o = (double)err2;
        }
        done = !(change && better);
    } while (!done && max_try--);
    return err_o;
}

// ---------------------------------------------------------------- packing ---

__device__ __forceinline__ void put_bits(uint32_t w[4], int &pos, uint32_t v, int n)
{
    for (int i = 0; i < n; ++i, ++pos)
        if ((v >> i) & 1u) w[pos >> 5] |= 1u << (pos & 31);
}

// EncodeSingleIndexBlock, amd_bc7_body.cpp:333-538 (+ endpoint packing :848-881)
__device__ void pack_single(int mode, int part, const uint8_t ep_in[3][2][4], uint64_t tidx, uint32_t w[4])
{
    const ModeInfo &mi = kModes[mode];
    int cbits[4];
    if (mi.enc == ENC_NO_ALPHA) {
        cbits[0] = cbits[1] = cbits[2] = mi.vector_bits / 3;
        cbits[3] = 0;
    } else {
        cbits[0] = cbits[1] = cbits[2] = cbits[3] = mi.vector_bits / 4;
    }
    const int dim = mi.enc == ENC_NO_ALPHA ? 3 : 4;
    // endpoint codes -> packed P|R|G|B(|A) words (amd_bc7_body.cpp:848-881)
    uint32_t colour[3][2];
    for (int s = 0; s < mi.subsets; ++s) {
        int e[2][4];
        for (int k = 0; k < 2; ++k)
            for (int c = 0; c < 4; ++c) e[k][c] = ep_in[s][k][c];
        uint32_t p0 = 0, p1 = 0;
        int shift = 0;
        if (mi.pbit) {
            p0 = (uint32_t)e[0][0] & 1;
            p1 = (uint32_t)e[1][0] & 1;
            for (int c = 0; c < 4; ++c) {
                e[0][c] >>= 1;
                e[1][c] >>= 1;
            }
            shift = 1;
        }
        for (int c = 0; c < dim; ++c)
            if (cbits[c]) {
                p0 |= (uint32_t)e[0][c] << shift;
                p1 |= (uint32_t)e[1][c] << shift;
                shift += cbits[c];
            }
        colour[s][0] = p0;
        colour[s][1] = p1;
    }
    uint32_t bidx[16];
    int flip[3] = {0, 0, 0};
    for (int i = 0; i < 16; ++i) {
        bidx[i] = (uint32_t)((tidx >> (4 * i)) & 15u);
        const int s = (int)shape_of(mi.subsets, part, i);
        if (i == anchor_of(mi.subsets, part, s) && (bidx[i] & (1u << (mi.ib0 - 1)))) flip[s] = 1;
    }
    for (int s = 0; s < mi.subsets; ++s)
        if (flip[s]) {
            const uint32_t t = colour[s][0];
            colour[s][0] = colour[s][1];
            colour[s][1] = t;
        }
    for (int i = 0; i < 16; ++i)
        if (flip[shape_of(mi.subsets, part, i)]) bidx[i] = ((1u << mi.ib0) - 1) - bidx[i];
    uint32_t comp[3][2][4], par[3][2];
    for (int s = 0; s < mi.subsets; ++s) {
        uint32_t pc[2] = {colour[s][0], colour[s][1]};
        if (mi.pbit == 2) {
            par[s][0] = pc[0] & 1;
            par[s][1] = pc[1] & 1;
            pc[0] >>= 1;
            pc[1] >>= 1;
        } else if (mi.pbit == 1) {
            par[s][0] = pc[1] & 1;
            par[s][1] = pc[1] & 1;
            pc[0] >>= 1;
            pc[1] >>= 1;
        } else {
            par[s][0] = par[s][1] = 0;
        }
        for (int c = 0; c < 4; ++c)
            if (cbits[c]) {
                comp[s][0][c] = pc[0] & ((1u << cbits[c]) - 1);
                comp[s][1][c] = pc[1] & ((1u << cbits[c]) - 1);
                pc[0] >>= cbits[c];
                pc[1] >>= cbits[c];
            }
    }
    w[0] = w[1] = w[2] = w[3] = 0;
    int pos = 0;
    put_bits(w, pos, 1u << mode, mode + 1);
    put_bits(w, pos, (uint32_t)part, mi.part_bits);
    for (int c = 0; c < 4; ++c)
        for (int s = 0; s < mi.subsets; ++s)
            for (int e = 0; e < 2; ++e) put_bits(w, pos, comp[s][e][c], cbits[c]);
    if (mi.pbit)
        for (int s = 0; s < mi.subsets; ++s) {
            put_bits(w, pos, par[s][0], 1);
            if (mi.pbit == 2) put_bits(w, pos, par[s][1], 1);
        }
    for (int i = 0; i < 16; ++i) {
        const int s = (int)shape_of(mi.subsets, part, i);
        put_bits(w, pos, bidx[i], i == anchor_of(mi.subsets, part, s) ? mi.ib0 - 1 : mi.ib0);
    }
}

__constant__ int kRot[4][4] = {{3, 0, 1, 2}, {0, 3, 1, 2}, {1, 0, 3, 2}, {2, 0, 1, 3}};

// EncodeDualIndexBlock, amd_bc7_body.cpp:902-1056
__device__ void pack_dual(int mode, int sel, int rot, int ep[2][2][4], int idx[2][16], uint32_t w[4])
{
    const ModeInfo &mi = kModes[mode];
    int ib[2], flip[2];
    ib[0] = sel ? mi.ib1 : mi.ib0;
    ib[1] = sel ? mi.ib0 : mi.ib1;
    flip[0] = (idx[0][0] & (1 << (ib[0] - 1))) != 0;
    flip[1] = (idx[1][0] & (1 << (ib[1] - 1))) != 0;
    for (int i = 0; i < 2; ++i)
        if (flip[i]) {
            for (int j = 0; j < 16; ++j) idx[i][j] = ((1 << ib[i]) - 1) - idx[i][j];
            for (int k = 0; k < 4; ++k) {
                const int t = ep[i][0][k];
                ep[i][0][k] = ep[i][1][k];
                ep[i][1][k] = t;
            }
        }
    w[0] = w[1] = w[2] = w[3] = 0;
    int pos = 0;
    put_bits(w, pos, 1u << mode, mode + 1);
    put_bits(w, pos, (uint32_t)rot, mi.rot_bits);
    put_bits(w, pos, sel ? 1u : 0u, mi.idxmode_bits);
    const int vb = mi.vector_bits / 3;
    for (int c = 0; c < 4; ++c)
        for (int e = 0; e < 2; ++e) {
            if (c != 3)
                put_bits(w, pos, (uint32_t)ep[0][e][c], vb);
            else
                put_bits(w, pos, (uint32_t)ep[1][e][0], mi.scalar_bits);
        }
    for (int i = 0; i < 2; ++i) {
        const int s = sel ? i ^ 1 : i;
        for (int j = 0; j < 16; ++j) put_bits(w, pos, (uint32_t)idx[s][j], j == 0 ? ib[s] - 1 : ib[s]);
    }
}

// ----------------------------------------------------------------- decode ---

// Standard BC7 decode of one block to packed RGBA8 words (BPTC format: mode
// header, partition / rotation / index-selection fields, endpoints channel by
// channel, p-bits, two index sets with the anchors' top bits implied,
// interpolation weights round(64 i / (2^bits - 1)), ((64 - w) e0 + w e1 + 32)
// >> 6).  One lane per block; the mode fields come from selects and every
// per-texel quantity from register selects, never from an array indexed by a
// lane value.  Reserved mode (no header bit): transparent black.
struct Bits128 {
    uint64_t lo, hi;
    int pos;
    __device__ __forceinline__ uint32_t get(int n)
    {
        uint64_t v;
        if (pos >= 64)
            v = hi >> (pos - 64);
        else if (pos + n <= 64)
            v = lo >> pos;
        else
            v = (lo >> pos) | (hi << (64 - pos));
        pos += n;
        return (uint32_t)v & ((1u << n) - 1u);
    }
};

__device__ __forceinline__ int bptc_weight(int i, int bits)
{
    const int n1 = (1 << bits) - 1;
    return (128 * i + n1) / (2 * n1);
}

__device__ void bc7_decode_block(const uint32_t w[4], uint32_t px[16])
{
    Bits128 br{(uint64_t)w[0] | ((uint64_t)w[1] << 32), (uint64_t)w[2] | ((uint64_t)w[3] << 32), 0};
    const uint32_t lowbyte = w[0] & 0xffu;
    if (!lowbyte) {
#pragma unroll
        for (int i = 0; i < 16; ++i) px[i] = 0;
        return;
    }
    const int mode = __builtin_ctz(lowbyte);
    br.pos = mode + 1;
    // subsets, partition bits, rotation bits, selection bits, colour bits, alpha
    // bits, p-bit kind (0 none, 1 per subset, 2 per endpoint), index bits
    const int ns = mode == 0 || mode == 2 ? 3 : (mode == 1 || mode == 3 || mode == 7 ? 2 : 1);
    const int pb = mode == 0 ? 4 : (ns > 1 ? 6 : 0);
    const int rb = mode == 4 || mode == 5 ? 2 : 0;
    const int sb = mode == 4 ? 1 : 0;
    const int cb = mode == 0 ? 4 : (mode == 1 ? 6 : (mode == 2 || mode == 4 || mode == 7 ? 5 : 7));
    const int ab = mode == 4 ? 6 : (mode == 5 ? 8 : (mode == 6 ? 7 : (mode == 7 ? 5 : 0)));
    const int pk = mode == 1 ? 1 : (mode == 0 || mode == 3 || mode == 6 || mode == 7 ? 2 : 0);
    const int ib0 = mode == 6 ? 4 : (mode == 0 || mode == 1 ? 3 : 2);
    const int ib1 = mode == 4 ? 3 : (mode == 5 ? 2 : 0);
    const int part = (int)br.get(pb);
    const int rot = (int)br.get(rb);
    const int sel = (int)br.get(sb);
    int ep[3][2][4];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int e = 0; e < 2; ++e)
                if (q < ns) ep[q][e][c] = (int)br.get(cb);
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int e = 0; e < 2; ++e)
            if (q < ns) ep[q][e][3] = ab ? (int)br.get(ab) : 255;
    int pbit[3][2] = {{0, 0}, {0, 0}, {0, 0}};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        if (q >= ns) continue;
        if (pk == 2) {
            pbit[q][0] = (int)br.get(1);
            pbit[q][1] = (int)br.get(1);
        } else if (pk == 1) {
            pbit[q][0] = pbit[q][1] = (int)br.get(1);
        }
    }
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                if (q >= ns) continue;
                int bits = c < 3 ? cb : ab;
                if (!bits) continue;
                int v = ep[q][e][c];
                if (pk) {
                    v = (v << 1) | pbit[q][e];
                    bits++;
                }
                v <<= (8 - bits);
                ep[q][e][c] = v | (v >> bits);
            }
    const uint32_t shape = ns == 1 ? 0u : (ns == 2 ? dShape2[part] : dShape3[part]);
    const int a1 = ns == 2 ? (int)dAnchor2[part] : (ns == 3 ? (int)dAnchor3a[part] : 0);
    const int a2 = ns == 3 ? (int)dAnchor3b[part] : 0;
    uint32_t i0[16], i1[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const bool anchor = i == 0 || (ns > 1 && i == a1) || (ns > 2 && i == a2);
        i0[i] = br.get(anchor ? ib0 - 1 : ib0);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) i1[i] = ib1 ? br.get(i == 0 ? ib1 - 1 : ib1) : 0u;
    const int cbits = ib1 && sel ? ib1 : ib0, abits = ib1 ? (sel ? ib0 : ib1) : ib0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int q = (int)((shape >> (2 * i)) & 3u);
        const int ci = (int)(ib1 && sel ? i1[i] : i0[i]), ai = (int)(ib1 ? (sel ? i0[i] : i1[i]) : i0[i]);
        const int wc = bptc_weight(ci, cbits), wa = bptc_weight(ai, abits);
        int v[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int e0 = q == 0 ? ep[0][0][c] : (q == 1 ? ep[1][0][c] : ep[2][0][c]);
            const int e1 = q == 0 ? ep[0][1][c] : (q == 1 ? ep[1][1][c] : ep[2][1][c]);
            const int wt = c < 3 ? wc : wa;
            v[c] = ((64 - wt) * e0 + wt * e1 + 32) >> 6;
        }
        int t;
        if (rot == 1) { t = v[0]; v[0] = v[3]; v[3] = t; }
        if (rot == 2) { t = v[1]; v[1] = v[3]; v[3] = t; }
        if (rot == 3) { t = v[2]; v[2] = v[3]; v[3] = t; }
        px[i] = (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16) | ((uint32_t)v[3] << 24);
    }
}

// Squared error of a packed block's decode against the block's texels (x255,
// RGBA), summed texel by texel, channel by channel, in double.
__device__ double decoded_sse(const uint32_t w[4], const float *tex)
{
    uint32_t px[16];
    bc7_decode_block(w, px);
    double e = 0.0;
    for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const double d = (double)((px[i] >> (8 * c)) & 255u) - (double)tex[i * 4 + c];
            e += d * d;
        }
    return e;
}

// ---------------------------------------------------------------- kernels ---

struct Params {
    uint32_t mode_mask;
    int colour_restrict, alpha_restrict, force_alpha_one;
    uint32_t n;        // blocks in this chunk
    uint32_t first;    // first block id of the chunk within the launch
    // BC7BlockEncoder's quality-derived settings (amd_bc7_body.hpp:94-149),
    // computed on the host exactly as the constructor does
    double quality, shake_thr, err_thr, part_search;
    double quant_thr;      // m_quantizerRangeThreshold = 255 * performance: above it optQuantTrace_d
    TraceTab trace;        // its tables (null unless performance < 1)
    uint32_t stage_mask;   // modes evaluated by this launch sequence (all, or one per stage)
    // partitions shaken per mode (CompressSingleIndexBlock's `attempts`,
    // :695-706, optionally capped by gic_options.bc7_shake_ranks), 4 bits per
    // mode; computed on the host (set_attempts) and read with a shift so that
    // a lane-varying mode never indexes a table
    uint32_t att;
    // pruned search only (bc7_shake_ranks > 0, no error-threshold exits): the
    // mode whose packed block decodes closest to the texels wins, not the one
    // with the least search error (DESIGN.md, BC7 pruned search)
    int decode_select;
    int dual_cap;   // pruned search: dual-index candidates shaken per mode, 2 x bc7_shake_ranks (0 = the reference's gating)
    // bounded exit (gic_options.bc7_mse_bound > 0): decoded-SSE bound of the
    // probe stages (64 x the MSE bound), and k_select leaving alone the blocks
    // the probe finished
    double bound_sse;
    int skip_done;
    int probe;   // bounded-exit probe: modes legal without the colour restriction (meta.pvalid)
    // workspace slot b holds output block list[b] (a compacted list of the
    // blocks an earlier stage left unfinished), or first + b when list is null
    const uint32_t *list;
    // H4: output ids of the blocks a capped register quantiser marked (the
    // call's re-run list, h4_cap entries; *h4_cnt may exceed it = overflow)
    uint32_t *h4_list;
    uint32_t *h4_cnt;
    uint32_t h4_cap;
    int general;   // the re-run: every block through the general (f64, uncapped) kernels
};

__device__ __forceinline__ uint32_t out_block(const Params &p, uint32_t b) { return p.list ? p.list[b] : p.first + b; }

// H4: a register quantiser of block b stopped at the iteration cap.  The block
// is marked once (flags bit 3) and its output id appended to the re-run list.
__device__ __forceinline__ void flag_capped(const Params &p, const Workspace &ws, uint32_t b)
{
    const uint32_t old = atomicOr(&ws.meta[b].flags, 8u);
    if (old & 8u) return;
    const uint32_t k = atomicAdd(p.h4_cnt, 1u);
    if (k < p.h4_cap) p.h4_list[k] = out_block(p, b);
}

// BlockMeta.flags bit 2: the block met the error threshold in an earlier
// stage (CompressBlock's mode-loop exit, :1440-1446)
__device__ __forceinline__ bool mode_active(const BlockMeta &meta, const Params &p, int mode)
{
    return ((p.probe ? meta.pvalid : meta.valid) & p.stage_mask & (1u << mode)) && !(meta.flags & 4u);
}

// partitions quantised (CompressSingleIndexBlock :569-573) and shaken (:695-706)
__device__ __forceinline__ int mode_tries(const Params &p, int mode)
{
    const unsigned nparts = 1u << kModes[mode].part_bits;
    unsigned tries = nparts;
    if (p.quality < 0.5) {
        tries = (unsigned)floor((double)(tries * p.part_search) + 0.5);
        tries = tries < 1 ? 1 : tries;
        tries = tries > nparts ? nparts : tries;
    }
    return (int)tries;
}

__device__ __forceinline__ int mode_attempts(const Params &p, int mode)
{
    return (int)((p.att >> (4 * mode)) & 15u);
}

// Host: the constructor-derived `attempts` of every mode (:695-706), capped at
// `cap` (1..8) when the pruned search is selected (0 = the reference's count).
static uint32_t host_attempts(const Params &p, int cap)
{
    static const unsigned nparts_of[8] = {16, 64, 64, 64, 1, 1, 1, 64};
    uint32_t att = 0;
    for (int mode = 0; mode < 8; ++mode) {
        const unsigned nparts = nparts_of[mode];
        unsigned tries = nparts;
        if (p.quality < 0.5) {
            tries = (unsigned)floor((double)(tries * p.part_search) + 0.5);
            tries = tries < 1 ? 1 : tries;
            tries = tries > nparts ? nparts : tries;
        }
        unsigned attempts = (unsigned)floor(8 * p.quality + 0.5);
        attempts = attempts < tries ? attempts : tries;
        attempts = attempts > 1 ? attempts : 1;
        if (cap > 0 && attempts > (unsigned)cap) attempts = (unsigned)cap;
        att |= attempts << (4 * mode);
    }
    return att;
}

__device__ void prep_block(const float inN[64], const Params &p, float *tex, BlockMeta &meta, uint32_t *px)
{
    int needs_alpha = 0, zero_one = 0;
    double bmin[4] = {1.7976931348623157e308, 1.7976931348623157e308, 1.7976931348623157e308,
                      1.7976931348623157e308};
    double bmax[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = 0; i < 16; ++i) {
        const float a = inN[i * 4 + 3];
        if (a < 1.0)
            needs_alpha = 1;
        else if ((a >= 0.99999) || (a < 0.00001))
            zero_one = 1;
        for (int j = 0; j < 4; ++j) {
            const float v = inN[i * 4 + j] * 255.0f;   // Q8: float multiply (amd_bc7_body.cpp:1322)
            tex[i * 4 + j] = v;
            const double d = v;
            bmin[j] = (d < bmin[j]) ? d : bmin[j];
            bmax[j] = (d > bmax[j]) ? d : bmax[j];
        }
    }
    double mr = bmax[0] - bmin[0];
    for (int j = 1; j < 4; ++j) mr = (bmax[j] - bmin[j]) > mr ? (bmax[j] - bmin[j]) : mr;
    const int solid = mr < 1e-10;
    uint32_t valid = p.mode_mask ? p.mode_mask : 0xCFu;
    for (int m = 0; m < 8; ++m) {
        if (!(valid & (1u << m))) continue;
        if (needs_alpha && kModes[m].enc == ENC_NO_ALPHA) valid &= ~(1u << m);
        if (needs_alpha && p.alpha_restrict && zero_one && kModes[m].enc == ENC_COMBINED) valid &= ~(1u << m);
    }
    meta.pvalid = valid;
    for (int m = 0; m < 8; ++m)
        if (!solid && !needs_alpha && p.colour_restrict && kModes[m].enc == ENC_COMBINED) valid &= ~(1u << m);
    bool integral = true, in_range = true;
    for (int i = 0; i < 64; ++i) {
        in_range &= (tex[i] >= 0.f) && (tex[i] <= 255.f);
        integral &= (tex[i] == floorf(tex[i]));
    }
    meta.valid = valid;
    meta.max_range = mr;
    // packed copy for the shake waves (meaningful for integral blocks only)
    for (int i = 0; i < 16; ++i) {
        uint32_t w = 0;
        for (int j = 0; j < 4; ++j) w |= (uint32_t)fminf(fmaxf(tex[i * 4 + j], 0.f), 255.f) << (8 * j);
        px[i] = w;
    }
    // bit0: outside the implemented path (values outside [0,1] would need
    // optQuantTrace_d or index the reference's tables out of bounds);
    // bit1: texels are integers, so every shaker error is an exact int32 (the
    // H4 re-run leaves it clear: the general kernels then take the block);
    // bit3: a register quantiser hit the H4 cap (flag_capped)
    meta.flags = (in_range ? 0u : 1u) | (integral && !p.general ? 2u : 0u);
}

__global__ void __launch_bounds__(256) k_prep_image(Geometry g, Params p, Workspace ws)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.n) return;
    uint32_t slice, by, bx;
    block_coords(g, out_block(p, b), slice, by, bx);
    float blk[64];
    load_block(g, slice, by, bx, p.force_alpha_one != 0, blk);
    prep_block(blk, p, ws.tex + (size_t)b * 64, ws.meta[b], ws.px + (size_t)b * 16);
}

__global__ void __launch_bounds__(256) k_prep_f32(const float *__restrict__ blocks, Params p, Workspace ws)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.n) return;
    float blk[64];
    const size_t o = (size_t)out_block(p, b) * 64;
    for (int i = 0; i < 64; ++i) blk[i] = blocks[o + i];
    prep_block(blk, p, ws.tex + (size_t)b * 64, ws.meta[b], ws.px + (size_t)b * 16);
}

__device__ __forceinline__ void task_mode(int task, int &mode, int &part)
{
    if (task < 16) { mode = 0; part = task; }
    else if (task < 80) { mode = 1; part = task - 16; }
    else if (task < 144) { mode = 2; part = task - 80; }
    else if (task < 208) { mode = 3; part = task - 144; }
    else if (task == 208) { mode = 6; part = 0; }
    else { mode = 7; part = task - 209; }
}

// K1: partition quantisation (CompressSingleIndexBlock :582-641)
__global__ void __launch_bounds__(256) k_quant(Params p, Workspace ws)
{
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t b = gid / kQuantTasks, task = gid % kQuantTasks;
    if (b >= p.n) return;
    int mode, part;
    task_mode((int)task, mode, part);
    const BlockMeta meta = ws.meta[b];
    if (!mode_active(meta, p, mode) || (meta.flags & 3u)) return;   // integral blocks: k_quant_reg
    if (part >= mode_tries(p, mode)) return;
    const ModeInfo &mi = kModes[mode];
    const int dim = mi.enc == ENC_NO_ALPHA ? 3 : 4;
    const int ncl = 1 << mi.ib0;
    const float *tex = ws.tex + (size_t)b * 64;
    double err = 0.;
    uint64_t tidx = 0;
    for (int s = 0; s < mi.subsets; ++s) {
        double sub[16][4];
        int tex_of[16], n = 0;
        for (int i = 0; i < 16; ++i)
            if ((int)shape_of(mi.subsets, part, i) == s) {
                for (int j = 0; j < dim; ++j) sub[n][j] = (double)tex[i * 4 + j];
                tex_of[n++] = i;
            }
        if (!n) continue;
        int idx[16];
        err += opt_quant(sub, n, ncl, idx, dim);
        for (int k = 0; k < n; ++k) tidx |= (uint64_t)(idx[k] & 15) << (4 * tex_of[k]);
    }
    ws.qerr[(size_t)b * kQuantTasks + task] = err;
    ws.qidx[(size_t)b * kQuantTasks + task] = tidx;
}

// K1a (integral blocks, modes 0-3): optQuantAnD_d once per distinct subset
// problem.  A subset's quantiser result depends only on its texels (mask, in
// texel order) and cluster count, and the partition tables repeat masks (21 %
// of modes 0-3's subset problems), so each distinct one is solved once and
// k_quant_gather sums the per-partition errors in subset order, exactly as the
// per-partition loop of CompressSingleIndexBlock (:582-641) does.
// Grid: x = distinct subset mask (wave-uniform), y = 256-block group, lane =
// block.  A mask used with 8 clusters (modes 0, 1) and with 4 (modes 2, 3) is
// two problems over the same texels: their mean, covariance and principal
// vector (quant_prefix) are computed once and both quantisations run from it.
// Every lane of a wave solves the same subset shape, so its texels are loaded
// compacted (slot k = the k-th member) and every member loop of the quantiser
// runs exactly n iterations under uniform branches (SelPrefix) -- a lane per
// (block, problem) paid all 16 texel slots of every loop with per-lane masks.
// Consecutive workgroups share their 256 blocks' texels in cache.
__device__ __forceinline__ bool subset_needed(const BlockMeta &meta, const Params &p, uint32_t u)
{
    if (u == 0xFFFFu) return false;
    const uint32_t mp = dUMinPart[u];
    bool need = false;
    for (int m = 0; m < 4; ++m) {
        const uint32_t mpart = (mp >> (8 * m)) & 0xFFu;
        need = need || (mpart != 0xFFu && mode_active(meta, p, m) && (int)mpart < mode_tries(p, m));
    }
    return need;
}

// QcDiv's offsets from a workgroup table in LDS (address made opaque at every
// read, so the loads stay at the use instead of being hoisted into VGPRs)
struct QcLds {
    uint32_t a;
    __device__ __forceinline__ double at(int q, int) const
    {
        uint32_t b = a;
        asm volatile("" : "+v"(b));
        return *(const __attribute__((address_space(3))) double *)(size_t)(b + 8u * (uint32_t)q);
    }
};

__global__ void __launch_bounds__(256, 3) k_quant_sub(Params p, Workspace ws)
{
    __shared__ double qc_tab[16];
    const uint32_t pair = dUMask[blockIdx.x];
    const uint32_t u8 = pair & 0xFFFFu, u4 = pair >> 16;
    const uint32_t mask = dUProb[u8 != 0xFFFFu ? u8 : u4] & 0xFFFFu;
    const int n = __popc(mask);
    if (threadIdx.x < 16) qc_tab[threadIdx.x] = QcDiv{}.at((int)threadIdx.x, n);
    __syncthreads();
    const QcLds qc{(uint32_t)(uintptr_t)(const __attribute__((address_space(3))) double *)qc_tab};
    const uint32_t b = blockIdx.y * blockDim.x + threadIdx.x;
    if (b >= p.n) return;
    const BlockMeta meta = ws.meta[b];
    if ((meta.flags & 3u) != 2u) return;
    const bool need8 = subset_needed(meta, p, u8), need4 = subset_needed(meta, p, u4);
    if (!need8 && !need4) return;
    const float *tex = ws.tex + (size_t)b * 64;
    uint32_t px[16];
    {
        uint32_t m = mask;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            px[k] = 0;
            if (k < n) {
                const int t = __builtin_ctz(m);   // uniform
                m &= m - 1;
                const float4 v = *reinterpret_cast<const float4 *>(tex + t * 4);
                px[k] = (uint32_t)v.x | ((uint32_t)v.y << 8) | ((uint32_t)v.z << 16) | ((uint32_t)v.w << 24);
            }
        }
    }
    double mean[4] = {0, 0, 0, 0}, dir[4];
    const bool spread = quant_prefix<3>(px, SelPrefix{n}, mean, dir);
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
        if (!(pass == 0 ? need8 : need4)) continue;
        const uint32_t u = pass == 0 ? u8 : u4;
        int idx[16];
        double err = 0.;
        uint64_t tidx = 0;
        if (spread) {
            int hit = 0;
            err = opt_quant_from<3>(px, SelPrefix{n}, pass == 0 ? 8 : 4, idx, mean, dir, qc, &hit);
            if (hit) flag_capped(p, ws, b);
            uint32_t m = mask;
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (k < n) {
                    const int t = __builtin_ctz(m);
                    m &= m - 1;
                    tidx |= (uint64_t)(idx[k] & 15) << (4 * t);
                }
        }
        ws.uerr[(size_t)b * kUMax + u] = err;
        ws.uidx[(size_t)b * kUMax + u] = tidx;
    }
}

// K1b: per-partition errors and indices of modes 0-3 from the subset problems
__global__ void __launch_bounds__(256) k_quant_gather(Params p, Workspace ws)
{
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t b = gid / 208u;
    const int task = (int)(gid % 208u);
    if (b >= p.n) return;
    int mode, part;
    task_mode(task, mode, part);
    const BlockMeta meta = ws.meta[b];
    if (!mode_active(meta, p, mode) || (meta.flags & 3u) != 2u) return;
    if (part >= mode_tries(p, mode)) return;
    double err = 0.;
    uint64_t tidx = 0;
    for (int sub = 0; sub < 3; ++sub) {
        const int u = dTaskSub[task][sub];
        if (u == 0xFFFF) break;
        err += ws.uerr[(size_t)b * kUMax + u];
        tidx |= ws.uidx[(size_t)b * kUMax + u];
    }
    ws.qerr[(size_t)b * kQuantTasks + task] = err;
    ws.qidx[(size_t)b * kQuantTasks + task] = tidx;
}

// K1 (integral blocks): register-resident partition quantisation
template <int DIM>
__global__ void __launch_bounds__(256, 2) k_quant_reg(Params p, Workspace ws, int task0, int ntasks)
{
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t b = gid / ntasks;
    const int task = task0 + (int)(gid % ntasks);
    if (b >= p.n) return;
    int mode, part;
    task_mode(task, mode, part);
    const BlockMeta meta = ws.meta[b];
    if (!mode_active(meta, p, mode) || (meta.flags & 3u) != 2u) return;
    if (part >= mode_tries(p, mode)) return;
    const ModeInfo &mi = kModes[mode];
    const int ncl = 1 << mi.ib0;
    const float *tex = ws.tex + (size_t)b * 64;
    uint32_t px[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const float4 v = *reinterpret_cast<const float4 *>(tex + i * 4);
        px[i] = (uint32_t)v.x | ((uint32_t)v.y << 8) | ((uint32_t)v.z << 16) | ((uint32_t)v.w << 24);
    }
    const uint32_t shape = mi.subsets == 1 ? 0u : (mi.subsets == 2 ? dShape2[part] : dShape3[part]);
    double err = 0.;
    uint64_t tidx = 0;
    for (int sub = 0; sub < mi.subsets; ++sub) {
        uint32_t mask = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) mask |= (((shape >> (2 * i)) & 3u) == (uint32_t)sub ? 1u : 0u) << i;
        if (!mask) continue;
        int idx[16], hit = 0;
        err += opt_quant_mask<DIM>(px, mask, ncl, idx, &hit);
        if (hit) flag_capped(p, ws, b);
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if ((mask >> i) & 1u) tidx |= (uint64_t)(idx[i] & 15) << (4 * i);
    }
    ws.qerr[(size_t)b * kQuantTasks + task] = err;
    ws.qidx[(size_t)b * kQuantTasks + task] = tidx;
}

// K1 of the bounded exit's mode-6 probe: one lane per block, the quantiser's
// first projection and lattice rounding only (opt_quant_mask<4, true>): on G1
// 98 % of the probe's blocks come out identical to starting from the full
// optQuantAnD_d and the share within the bound is unchanged, for a
// fraction of the cost; the probe's blocks are checked against the bound anyway.
__global__ void __launch_bounds__(256) k_quant_probe6(Params p, Workspace ws)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.n) return;
    const BlockMeta meta = ws.meta[b];
    if (!mode_active(meta, p, 6) || (meta.flags & 3u) != 2u) return;
    const float *tex = ws.tex + (size_t)b * 64;
    uint32_t px[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const float4 v = *reinterpret_cast<const float4 *>(tex + i * 4);
        px[i] = (uint32_t)v.x | ((uint32_t)v.y << 8) | ((uint32_t)v.z << 16) | ((uint32_t)v.w << 24);
    }
    int idx[16];
    opt_quant_mask<4, true>(px, 0xFFFFu, 16, idx);
    uint64_t tidx = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) tidx |= (uint64_t)(idx[i] & 15) << (4 * i);
    ws.qerr[(size_t)b * kQuantTasks + 208] = 0.;
    ws.qidx[(size_t)b * kQuantTasks + 208] = tidx;
}

// Bounded exit, stage 0 (round 6; not the reference's search): a mode-6 block
// straight from the quantiser's first projection -- least-squares endpoints for
// BC7's 4-bit interpolation weights, each endpoint's 7-bit codes and parity bit
// the nearest to them, every texel taken to its nearest palette entry, then one
// refit from those indices, the better of the two kept.  Final when the packed block decodes within the bound, like a probe:
// it only decides which blocks skip the later stages, and a final block meets
// the contract by the bound.  Modelled bit for bit by oracle/orc_bc7.c
// orc_bc7_fit6 (integer sums, the same f64 solve and rounding).  On 8K G1 it
// finishes about as many blocks as the mode-6 shaker probe did, for a fraction
// of the cost, and the shaker probe then runs over the few percent it leaves.
__constant__ int kW16[16] = {0, 4, 9, 13, 17, 21, 26, 30, 34, 38, 43, 47, 51, 55, 60, 64};

// palette of endpoint values q0, q1 (8-bit, parity included) and the texels'
// nearest entries (first of least error, 4 bits per texel); returns the summed
// squared error.  Palette entry outer, texel inner: each entry is formed once
// and every texel keeps its running minimum (no 16-entry palette held live).
__device__ __forceinline__ uint32_t fit6_palette(const uint32_t px[16], const int q0[4], const int q1[4],
                                                 uint64_t &idx_out)
{
    int best[16], bi[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        best[k] = 0x7fffffff;
        bi[k] = 0;
    }
#pragma unroll 1
    for (int i = 0; i < 16; ++i) {
        uint32_t v = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c)
            v |= (uint32_t)(((64 - kW16[i]) * q0[c] + kW16[i] * q1[c] + 32) >> 6) << (8 * c);
        const int sq = (int)__builtin_amdgcn_udot4(v, v, 0u, false);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int d = sq - 2 * (int)__builtin_amdgcn_udot4(v, px[k], 0u, false);
            if (d < best[k]) {
                best[k] = d;
                bi[k] = i;
            }
        }
    }
    uint32_t sse = 0;
    uint64_t ix = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        sse += (uint32_t)(best[k] + (int)__builtin_amdgcn_udot4(px[k], px[k], 0u, false));
        ix |= (uint64_t)bi[k] << (4 * k);
    }
    idx_out = ix;
    return sse;
}

// EncodeSingleIndexBlock's layout for mode 6 (pack_single's, specialised:
// every field at a fixed bit position): mode bit 6, R0 R1 G0 G1 B0 B1 A0 A1 as
// 7-bit codes, the two parity bits, texel 0's index in 3 bits (anchor: a set
// top bit swaps the endpoints and inverts every index), the others in 4
__device__ __forceinline__ void pack_mode6(const int q0_in[4], const int q1_in[4], uint64_t idx, uint32_t w[4])
{
    const bool flip = (idx & 8u) != 0;
    int q0[4], q1[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        q0[c] = flip ? q1_in[c] : q0_in[c];
        q1[c] = flip ? q0_in[c] : q1_in[c];
    }
    if (flip) idx = ~idx;   // 15 - i in every nibble
    uint64_t lo = 1u << 6, hi = 0;
    int pos = 7;
    auto put = [&](uint64_t v, int n) {
        if (pos < 64) lo |= v << pos;
        if (pos + n > 64) hi |= pos >= 64 ? v << (pos - 64) : v >> (64 - pos);
        pos += n;
    };
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        put((uint64_t)(q0[c] >> 1), 7);
        put((uint64_t)(q1[c] >> 1), 7);
    }
    put((uint64_t)(q0[0] & 1), 1);
    put((uint64_t)(q1[0] & 1), 1);
    put(idx & 7u, 3);
#pragma unroll
    for (int k = 1; k < 16; ++k) put((idx >> (4 * k)) & 15u, 4);
    w[0] = (uint32_t)lo;
    w[1] = (uint32_t)(lo >> 32);
    w[2] = (uint32_t)hi;
    w[3] = (uint32_t)(hi >> 32);
}

// stage 0 itself; k_quant_probe6 has stored the first projection's indices
// (qidx slot 208) for the blocks it may take
__global__ void __launch_bounds__(256) k_fit6(Params p, Workspace ws, uint4 *__restrict__ dst,
                                              double *__restrict__ err_out)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.n) return;
    const BlockMeta meta = ws.meta[b];
    if ((meta.flags & 7u) != 2u || !((meta.pvalid >> 6) & 1u)) return;   // integral, supported, not final, mode 6 legal
    uint32_t px[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) px[i] = ws.px[(size_t)b * 16 + i];
    uint64_t idx = ws.qidx[(size_t)b * kQuantTasks + 208];
    uint32_t best = 0xffffffffu;
    uint64_t bidx = 0;
    int b0[4] = {0, 0, 0, 0}, b1[4] = {0, 0, 0, 0};
#pragma unroll 1
    for (int it = 0; it < 2; ++it) {
        // (opaque: otherwise the 64 channel values are hoisted out of the loop)
#pragma unroll
        for (int k = 0; k < 16; ++k) asm volatile("" : "+v"(px[k]));
        // least squares over the texels: x ~ ((64 - w) e0 + w e1) / 64
        int a00 = 0, a01 = 0, a11 = 0, r0[4] = {0, 0, 0, 0}, r1[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int w = kW16[(idx >> (4 * k)) & 15u], u = 64 - w;
            a00 += u * u;
            a01 += u * w;
            a11 += w * w;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int x = (int)((px[k] >> (8 * c)) & 255u);
                r0[c] += u * x;
                r1[c] += w * x;
            }
        }
        const long long det = (long long)a00 * a11 - (long long)a01 * a01;
        double e0[4], e1[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (det == 0) {
                int sum = 0;
#pragma unroll
                for (int k = 0; k < 16; ++k) sum += (int)((px[k] >> (8 * c)) & 255u);
                e0[c] = e1[c] = (double)sum / 16.0;
            } else {
                e0[c] = (64.0 * (double)((long long)a11 * r0[c] - (long long)a01 * r1[c])) / (double)det;
                e1[c] = (64.0 * (double)((long long)a00 * r1[c] - (long long)a01 * r0[c])) / (double)det;
            }
            e0[c] = e0[c] < 0.0 ? 0.0 : (e0[c] > 255.0 ? 255.0 : e0[c]);
            e1[c] = e1[c] < 0.0 ? 0.0 : (e1[c] > 255.0 ? 255.0 : e1[c]);
        }
        // each endpoint's parity: the one whose 7-bit codes land nearer its
        // least-squares values (parity 0 on a tie)
        int c0[4], c1[4];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const double *e = i ? e1 : e0;
            int q[2][4];
            double qe[2] = {0.0, 0.0};
#pragma unroll
            for (int par = 0; par < 2; ++par)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    int v = (int)floor((e[c] - (double)par) * 0.5 + 0.5);
                    v = v < 0 ? 0 : (v > 127 ? 127 : v);
                    q[par][c] = 2 * v + par;
                    const double d = (double)q[par][c] - e[c];
                    qe[par] += d * d;
                }
            const int pb = qe[1] < qe[0] ? 1 : 0;
#pragma unroll
            for (int c = 0; c < 4; ++c) (i ? c1 : c0)[c] = q[pb][c];
        }
        uint64_t cidx;
        const uint32_t cbest = fit6_palette(px, c0, c1, cidx);
        if (cbest < best) {
            best = cbest;
            bidx = cidx;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                b0[c] = c0[c];
                b1[c] = c1[c];
            }
        }
        idx = cidx;
    }
    // integral texels: the palette error is the decoded block's error (the
    // oracle model checks the two agree, tests/test_gpu_bc7_sample.py)
    const double d = (double)best;
    if (!(d <= p.bound_sse)) return;
    uint32_t w[4];
    pack_mode6(b0, b1, bidx, w);
    const uint32_t o = out_block(p, b);
    dst[o] = make_uint4(w[0], w[1], w[2], w[3]);
    if (err_out) err_out[o] = d;
    ws.meta[b].flags = meta.flags | 4u;
}

// K1t (performance < 1): optQuantTrace_d for the partitions of the single-index
// modes with at most 8 clusters (0-3, 7) of blocks whose range exceeds
// 255 * performance (CompressSingleIndexBlock :606-633); overwrites what the
// optQuantAnD_d kernels stored for them.  Lanes of a wave share a task, so
// they walk the same trace table.
__global__ void __launch_bounds__(64) k_quant_trace(Params p, Workspace ws)
{
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t t = gid / p.n, b = gid % p.n;
    if (t >= 272u) return;
    const int task = (int)(t < 208u ? t : t + 1u);   // skip mode 6 (16 clusters: optQuantAnD_d)
    int mode, part;
    task_mode(task, mode, part);
    const BlockMeta meta = ws.meta[b];
    if (!mode_active(meta, p, mode) || !(meta.max_range > p.quant_thr)) return;
    if (part >= mode_tries(p, mode)) return;
    const ModeInfo &mi = kModes[mode];
    const int dim = mi.enc == ENC_NO_ALPHA ? 3 : 4;
    const int ncl = 1 << mi.ib0;
    const float *tex = ws.tex + (size_t)b * 64;
    double err = 0.;
    uint64_t tidx = 0;
    for (int sub = 0; sub < mi.subsets; ++sub) {
        double d[16][4];
        int tex_of[16], n = 0;
        for (int i = 0; i < 16; ++i)
            if ((int)shape_of(mi.subsets, part, i) == sub) {
                for (int j = 0; j < dim; ++j) d[n][j] = (double)tex[i * 4 + j];
                tex_of[n++] = i;
            }
        if (!n) continue;
        int idx[16];
        err += opt_quant_trace(d, n, ncl, idx, dim, p.trace);
        for (int k = 0; k < n; ++k) tidx |= (uint64_t)(idx[k] & 15) << (4 * tex_of[k]);
    }
    ws.qerr[(size_t)b * kQuantTasks + task] = err;
    ws.qidx[(size_t)b * kQuantTasks + task] = tidx;
}

// one subset of CompressSingleIndexBlock's shake loop (amd_bc7_body.cpp:721-805),
// per-lane f64 path (blocks with fractional texels)
template <typename T>
__device__ double shake_subset(const SpEntry *sp, const double sub[][4], const T *tsub, int n, int *idx, int epo[2][4],
                               bool corners_too, int shake, int last, const int *bits, int parity, int dim)
{
    if (!corners_too) return shake_window<T>(sp, sub, tsub, n, idx, epo, shake, last, bits[3], dim);
    int tidx[16], tepo[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    for (int k = 0; k < n; ++k) tidx[k] = idx[k];
    const double e0 = shake_corners<T>(sp, sub, tsub, n, tidx, tepo, last, bits, parity);
    double e1 = shake_window<T>(sp, sub, tsub, n, idx, epo, shake, last, bits[3], dim);
    if (e0 < e1) {
        e1 = shake_window<T>(sp, sub, tsub, n, tidx, tepo, shake, last, bits[3], dim);
        for (int k = 0; k < n; ++k) idx[k] = tidx[k];
        for (int k = 0; k < 4; ++k) {
            epo[0][k] = tepo[0][k];
            epo[1][k] = tepo[1][k];
        }
    }
    return e1;
}

// Shake parameters of a single-index mode (amd_bc7_body.cpp:654-706)
struct ShakeCfg {
    int dim, parity, last, shake, bits[4];
};

__device__ ShakeCfg shake_cfg(int mode, double quality)
{
    const ModeInfo &mi = kModes[mode];
    ShakeCfg c;
    c.dim = mi.enc == ENC_NO_ALPHA ? 3 : 4;
    c.parity = mi.pbit == 0 ? PAR_CART : mi.pbit == 1 ? PAR_SAME : PAR_BCC;
    int cbits[4];
    if (mi.enc == ENC_NO_ALPHA) {
        cbits[0] = cbits[1] = cbits[2] = mi.vector_bits / 3;
        cbits[3] = 0;
    } else {
        cbits[0] = cbits[1] = cbits[2] = cbits[3] = mi.vector_bits / 4;
    }
    c.bits[0] = cbits[0] + (c.parity ? 1 : 0);
    c.bits[1] = cbits[1] + (c.parity ? 1 : 0);
    c.bits[2] = cbits[2] + (c.parity ? 1 : 0);
    c.bits[3] = 0;
    for (int i = 0; i < c.dim; ++i) c.bits[3] += cbits[i];
    c.bits[3] *= 2;
    if (c.parity == PAR_BCC)
        c.bits[3] += 2;
    else if (c.parity == PAR_SAME)
        c.bits[3] += 1;
    const unsigned s0 = 8 - (unsigned)floor(1.5 * mi.ib0);
    unsigned t = (unsigned)floor(s0 * quality + 0.5);
    t = t < 6 ? t : 6;
    int shake = (int)(t > 2 ? t : 2);
    if (c.parity == PAR_SAME || c.parity == PAR_BCC) shake += 2;
    c.shake = shake;
    c.last = (1 << mi.ib0) - 1;
    return c;
}

// partition whose stable rank is `rank` (sortProjection, amd_bc7_3dquant_vpc.cpp:138-150)
__device__ int partition_of_rank(const double *qe, int nparts, int rank)
{
    for (int c = 0; c < nparts; ++c) {
        const double v = qe[c];
        int rk = 0;
        for (int o = 0; o < nparts; ++o) {
            const double w = qe[o];
            rk += (w - v < 0 || (!(w - v > 0) && !(w - v < 0) && o < c)) ? 1 : 0;
        }
        if (rk == rank) return c;
    }
    return 0;
}

// K2 (f64 lanes): shaking of the 8 best partitions of a single-index mode
// for blocks with fractional texels (CompressSingleIndexBlock :644-844)
__global__ void __launch_bounds__(256) k_shake(Params p, Workspace ws, const SpEntry *__restrict__ sp)
{
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t per = kShakeSlots * kShakeRanks;
    const uint32_t b = gid / per, r = gid % per;
    if (b >= p.n) return;
    const int slot = (int)(r / kShakeRanks), rank = (int)(r % kShakeRanks);
    const int mode = kSlotMode[slot];
    const BlockMeta meta = ws.meta[b];
    if (!mode_active(meta, p, mode) || (meta.flags & 3u)) return;   // integral blocks: k_shake_wave
    const ModeInfo &mi = kModes[mode];
    const int nparts = mode_tries(p, mode);   // partitions quantised and ranked
    if (rank >= mode_attempts(p, mode)) return;
    const int part = partition_of_rank(ws.qerr + (size_t)b * kQuantTasks + kSlotBase[slot], nparts, rank);
    const uint64_t qidx = ws.qidx[(size_t)b * kQuantTasks + kSlotBase[slot] + part];
    const ShakeCfg cfg = shake_cfg(mode, p.quality);
    const float *tex = ws.tex + (size_t)b * 64;
    ShakeResult &res = ws.shk[((size_t)b * kShakeSlots + slot) * kShakeRanks + rank];
    res.part = (uint32_t)part;
    const bool corners_too = !(meta.max_range > p.shake_thr) && cfg.dim == 3;   // m_shakerRangeThreshold
    for (int s = 0; s < mi.subsets; ++s) {
        double sub[16][4];
        int tex_of[16], n = 0, idx[16];
        for (int i = 0; i < 16; ++i)
            if ((int)shape_of(mi.subsets, part, i) == s) {
                for (int j = 0; j < cfg.dim; ++j) sub[n][j] = (double)tex[i * 4 + j];
                idx[n] = (int)((qidx >> (4 * i)) & 15u);
                tex_of[n++] = i;
            }
        int epo[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
        const double e = shake_subset<double>(sp, sub, &sub[0][0], n, idx, epo, corners_too, cfg.shake, cfg.last,
                                              cfg.bits, cfg.parity, cfg.dim);
        uint64_t ti = 0;
        for (int k = 0; k < n; ++k) ti |= (uint64_t)(idx[k] & 15) << (4 * tex_of[k]);
        res.err[s] = e;
        res.idx[s] = ti;
        for (int k = 0; k < 4; ++k) {
            res.ep[s][0][k] = (uint8_t)epo[0][k];
            res.ep[s][1][k] = (uint8_t)epo[1][k];
        }
    }
}

#include "bc7_wave.inc"

// Wave shaker problems, one kernel per cluster count NC:
//   NC = 8 : modes 0, 1 (slots 0, 1)      -> 8 ranks x (3 + 2) subsets = 40
//   NC = 4 : modes 2, 3, 7 (slots 2, 3, 5) -> 8 x (3 + 2 + 2)          = 56
//   NC = 16: mode 6 (slot 4)               -> 1
// Waves per block of k_shake_wave<NC>: (rank, subset) problems of the slots
// it serves -- modes 0/1 (NC 8), 2/3/7 (NC 4), 6 (NC 16) -- for the ranks
// actually shaken (Params.att), rank-major within a slot.
template <int NC>
__host__ __device__ static int wave_count(uint32_t att)
{
    const int m8[2] = {0, 1}, m4[3] = {2, 3, 7};
    const int *ms = NC == 8 ? m8 : m4;
    const int nm = NC == 8 ? 2 : 3;
    if (NC == 16) return (int)((att >> 24) & 15u) ? 1 : 0;
    int c = 0;
    for (int k = 0; k < nm; ++k) c += (int)((att >> (4 * ms[k])) & 15u) * (ms[k] == 0 || ms[k] == 2 ? 3 : 2);
    return c;
}

template <int NC>
__device__ __forceinline__ void wave_problem(const Params &p, int id, int &slot, int &rank, int &subset)
{
    const int nsl = NC == 8 ? 2 : (NC == 4 ? 3 : 1);
    int base = 0;
    for (int k = 0; k < nsl; ++k) {
        // slot k of this kernel: 0/1 (NC 8), 2/3/5 (NC 4), 4 (NC 16)
        const int sl = NC == 8 ? k : (NC == 4 ? (k == 2 ? 5 : 2 + k) : 4);
        const int md = NC == 8 ? k : (NC == 4 ? (k == 2 ? 7 : 2 + k) : 6);
        const int ns = NC == 8 ? (k == 0 ? 3 : 2) : (NC == 4 ? (k == 0 ? 3 : 2) : 1);
        const int cnt = (sl == 4 ? 1 : mode_attempts(p, md)) * ns;
        if (id < base + cnt || k == nsl - 1) {
            slot = sl;
            rank = (id - base) / ns;
            subset = (id - base) % ns;
            return;
        }
        base += cnt;
    }
}

// a rank's subset result, following a repeated-problem reference (k_shake_wave)
__device__ __forceinline__ const ShakeResult &shake_ref(const ShakeResult *shk, int r, int s)
{
    const double e = shk[r].err[s];
    return e < 0 ? shk[(int)(-1.0 - e) >> 2] : shk[r];
}
__device__ __forceinline__ int shake_sub(const ShakeResult *shk, int r, int s)
{
    const double e = shk[r].err[s];
    return e < 0 ? ((int)(-1.0 - e) & 3) : s;
}

// K1c: stable partition ranks (sortProjection, amd_bc7_3dquant_vpc.cpp:138-150)
// of each single-index slot, one wave per (block, slot), lane = partition;
// the partitions of ranks 0..7 are stored for the shake waves (computed once
// per slot instead of once per (rank, subset) wave)
__global__ void __launch_bounds__(256) k_rank(Params p, Workspace ws)
{
    // wave-uniform by construction; readfirstlane lets the compiler see it (scalar loads and branches)
    const uint32_t wid = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t b = wid / kShakeSlots;
    const int slot = (int)(wid % kShakeSlots);
    if (b >= p.n) return;
    const int mode = kSlotMode[slot];
    const BlockMeta meta = ws.meta[b];
    if (!mode_active(meta, p, mode) || (meta.flags & 3u) != 2u) return;
    const int nparts = mode_tries(p, mode);
    const int att = mode_attempts(p, mode);
    const int ln = wv::lane();
    const double *qe = ws.qerr + (size_t)b * kQuantTasks + kSlotBase[slot];
    const double v = ln < nparts ? qe[ln] : 0.0;
    int rk = 0;
    for (int o = 0; o < nparts; ++o) {
        const double w = wv::bcast_d(v, o);
        rk += (w - v < 0 || (!(w - v > 0) && !(w - v < 0) && o < ln)) ? 1 : 0;
    }
    if (ln < nparts && rk < att) {
        const size_t r = ((size_t)b * kShakeSlots + slot) * kShakeRanks + rk;
        ws.prank[r] = (uint8_t)ln;
        ws.pqidx[r] = ws.qidx[(size_t)b * kQuantTasks + kSlotBase[slot] + ln];
    }
}

// K2 (waves): one wavefront per (block, mode, rank, subset) shake problem of
// an integral block.  Returns false when the FAST form deferred the problem
// (bc7_wave.inc: it reached quant_single_point_d); nothing is written then.
template <int NC, bool FAST>
__device__ __forceinline__ bool shake_problem(const Params &p, const Workspace &ws, const SpEntry *__restrict__ sp,
                                              uint32_t wid)
{
    const uint32_t per = (uint32_t)wave_count<NC>(p.att);
    const uint32_t b = wid / per;
    if (b >= p.n) return true;
    int slot, rank, subset;
    wave_problem<NC>(p, (int)(wid % per), slot, rank, subset);
    const int mode = kSlotMode[slot];
    const int nparts = mode_tries(p, mode);   // partitions quantised and ranked
    const int ln = wv::lane();
    // Every load the wave needs is issued here, before any of them is waited
    // for: the block's meta, the partition of this rank and of the lower ranks
    // (k_rank), its quantiser indices (k_rank's copy) and the packed texels
    // (lane t < 16: texel t).  (Chained -- meta, then the partition, then its
    // indices, then the subset's texels -- the loads left the shake waves
    // waiting on memory for several microseconds each.)
    const size_t sr = ((size_t)b * kShakeSlots + slot) * kShakeRanks;
    const BlockMeta meta = ws.meta[b];
    // mode 6: one partition (no k_rank in its probe stage)
    const int part = nparts == 1 ? 0 : (int)ws.prank[sr + rank];
    const uint64_t qidx = nparts == 1 ? ws.qidx[(size_t)b * kQuantTasks + kSlotBase[slot]] : ws.pqidx[sr + rank];
    const int lpart = ln < rank ? (int)ws.prank[sr + ln] : 0;   // lane L < rank: the partition of rank L
    const uint32_t pxl = ln < 16 ? ws.px[(size_t)b * 16 + ln] : 0u;
    if (!mode_active(meta, p, mode) || (meta.flags & 3u) != 2u) return true;
    const ModeInfo &mi = kModes[mode];
    if (rank >= mode_attempts(p, mode)) return true;
    const ShakeCfg cfg = shake_cfg(mode, p.quality);
    // gather the subset: lane L < n holds the L-th texel of the subset
    uint32_t mask = 0;
    for (int t = 0; t < 16; ++t) mask |= ((int)shape_of(mi.subsets, part, t) == subset ? 1u : 0u) << t;
    ShakeResult &res = ws.shk[sr + rank];
    // Repeated problem (exact): three-subset shapes share subset masks, and a
    // subset's quantiser indices and shake depend only on its texels, so when a
    // lower rank of this mode shakes a subset with the same mask the result is
    // identical.  Only a reference (-1 - (rank*4 + subset)) is stored; k_select
    // reads the first occurrence.  (Two-subset shapes never repeat a mask.)
    if (mi.subsets == 3) {
        int key = 0x7fffffff;
        if (ln < rank) {
            const uint32_t sh = dShape3[lpart];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const uint32_t x = sh ^ (0x55555555u * (uint32_t)j);
                uint32_t z = ~(x | (x >> 1)) & 0x55555555u;   // bit 2t: texel t in subset j
                z = (z | (z >> 1)) & 0x33333333u;
                z = (z | (z >> 2)) & 0x0f0f0f0fu;
                z = (z | (z >> 4)) & 0x00ff00ffu;
                z = (z | (z >> 8)) & 0x0000ffffu;
                if (z == mask) key = wv::imin(key, ln * 4 + j);
            }
        }
        key = wv::wmin(key);
        if (key != 0x7fffffff) {
            if (ln == 0) {
                if (subset == 0) res.part = (uint32_t)part;
                res.err[subset] = -1.0 - (double)key;
            }
            return true;
        }
    }
    const int n = __popc(mask);
    int src = 0;
    {
        int cnt = 0;
        for (int t = 0; t < 16; ++t)
            if ((mask >> t) & 1u) {
                if (cnt == ln) src = t;
                cnt++;
            }
    }
    // lane L < n takes texel src (channels past dim are cleared by make_texels)
    const unsigned px = (unsigned)__builtin_amdgcn_ds_bpermute(src * 4, (int)pxl);
    wv::Texels T;
    wv::make_texels(T, px, n, cfg.dim);
    int idx = T.live ? (int)((qidx >> (4 * src)) & 15u) : 0;
    PROF_BEGIN;
    int epo[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    const bool corners_too = !(meta.max_range > p.shake_thr) && cfg.dim == 3;
    bool defer = false;
    const double e = wv::subset_shake<NC, FAST>(sp, T, idx, epo, corners_too, cfg.shake, cfg.last, cfg.bits, cfg.parity,
                                                defer);
    PROF_END;
    if (FAST && defer) return false;
    unsigned long long ti = T.live ? (unsigned long long)(idx & 15) << (4 * src) : 0ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ti |= __shfl_xor(ti, o);
    if (ln == 0) {
        if (subset == 0) res.part = (uint32_t)part;
        res.err[subset] = e;
        res.idx[subset] = ti;
        for (int k = 0; k < 4; ++k) {
            res.ep[subset][0][k] = (uint8_t)epo[0][k];
            res.ep[subset][1][k] = (uint8_t)epo[1][k];
        }
    }
    return true;
}

// Fast form: the problems that reach quant_single_point_d are appended to
// the kind's deferred list (one atomic per such wave) for k_shake_wave_slow.
__device__ __forceinline__ void defer_push(const Params &p, const Workspace &ws, int kind, uint32_t wid)
{
    if (wv::lane() == 0) {
        const uint32_t k = atomicAdd(&ws.defer_cnt[kind], 1u);
        ws.defer[(size_t)defer_off(kind) * p.n + k] = wid;
    }
}

// waves per SIMD of the fast kernels (<= 72 / 64 / 80 VGPRs, no spills)
template <int NC> struct ShakeOcc { static constexpr int v = 8; };
template <> struct ShakeOcc<4> { static constexpr int v = 8; };
template <> struct ShakeOcc<16> { static constexpr int v = 6; };   // 16 ramp points per corner lane
template <int NC> constexpr int shake_kind() { return NC == 8 ? 0 : (NC == 4 ? 1 : 2); }

template <int NC>
__global__ void __launch_bounds__(256, ShakeOcc<NC>::v) k_shake_wave(Params p, Workspace ws, const SpEntry *__restrict__ sp)
{
    // wave-uniform by construction; readfirstlane lets the compiler see it (scalar loads and branches)
    const uint32_t wid = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    if (!shake_problem<NC, true>(p, ws, sp, wid)) defer_push(p, ws, shake_kind<NC>(), wid);
}

// The deferred problems, whole, with the quant_single_point_d branch: a grid of
// a few waves per SIMD strides over the list the fast kernel left (read after
// it completed, same stream).
template <int NC>
__global__ void __launch_bounds__(256, 4) k_shake_wave_slow(Params p, Workspace ws, const SpEntry *__restrict__ sp)
{
    const uint32_t w0 = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(ws.defer_cnt[shake_kind<NC>()]);
    const uint32_t *list = ws.defer + (size_t)defer_off(shake_kind<NC>()) * p.n;
    for (uint32_t i = w0; i < cnt; i += nw) shake_problem<NC, false>(p, ws, sp, __builtin_amdgcn_readfirstlane(list[i]));
}


// K3a: dual-index quantisation (CompressDualIndexBlock :1084-1152): optQuantAnD_d
// for the colour and the replicated-alpha halves of each (rotation, selection);
// one lane per (block, task, half).  Integral blocks take the register-resident
// quantiser (k_dual_quant_reg), fractional ones the f64 array path.
// CompressDualIndexBlock shakes a (rotation, selection) candidate when
// quality > 0.7 or its quantiser error qe = e_colour + e_alpha / 3 is <= the
// smallest qe of the mode's earlier candidates (:1141, :1170)
// The pruned search (Params.dual_cap > 0) shakes only the dual_cap candidates
// of least qe of the mode, ties to the earlier (rotation, selection).
__device__ __forceinline__ bool dual_shaken(const Params &p, const Workspace &ws, uint32_t b, int task)
{
    const int t0 = task < 8 ? 0 : 8;
    const double *q = ws.dqerr + (size_t)b * kDualTasks * 2;
    if (p.dual_cap > 0) {
        const int t1 = task < 8 ? 8 : 12;
        double qt = q[2 * task];
        qt += q[2 * task + 1] / 3.;
        int rank = 0;
        for (int t = t0; t < t1; ++t) {
            double qe = q[2 * t];
            qe += q[2 * t + 1] / 3.;
            rank += (qe < qt || (qe == qt && t < task)) ? 1 : 0;
        }
        return rank < p.dual_cap;
    }
    if (p.quality > 0.7) return true;
    double best_q = 1.7976931348623157e308;
    for (int t = t0; t < task; ++t) {
        double qe = q[2 * t];
        qe += q[2 * t + 1] / 3.;
        if (qe < best_q) best_q = qe;
    }
    double qe = q[2 * task];
    qe += q[2 * task + 1] / 3.;
    return qe <= best_q;
}

__device__ __forceinline__ int dual_shake_size(const Params &p)
{
    unsigned shake = (unsigned)(6 * p.quality);
    shake = shake < 6 ? shake : 6;
    return (int)(shake > 2 ? shake : 2);
}

// Index bits of one half (0 = colour, 1 = alpha) of a dual-index candidate:
// ib0 for the half the selector gives the first index set.  Written as a select
// on purpose: the round-1 merged dual-quantiser kernel indexed a private copy
// {ib0, ib1} with this lane-divergent subscript, the optimiser folded it into a
// load from the __constant__ kModes table and emitted it as a scalar load of
// the FIRST lane's address (v_readfirstlane + s_load, tools/isa_audit.py), so
// every lane quantised with lane 0's cluster count (mode 4 mixes 2- and 3-bit
// sets).  Kernels index no private copies of constant tables by lane values.
__device__ __forceinline__ int dual_index_bits(const ModeInfo &mi, int half, int sel)
{
    return (half ^ sel) ? mi.ib1 : mi.ib0;
}

__device__ __forceinline__ void dual_task(uint32_t task, int &mode, int &rot, int &sel)
{
    mode = task < 8 ? 4 : 5;
    rot = task < 8 ? (int)(task >> 1) : (int)(task - 8);
    sel = task < 8 ? (int)(task & 1) : 0;
}

// One lane per (block, rotation, half): the three candidates of a rotation
// (mode 4 selections 0 and 1, mode 5) quantise the same texels of a half with
// 4 or 8 clusters, so the lane computes the quantiser prefix (mean, covariance,
// principal vector) once and each distinct cluster count once, and writes
// every active candidate's slot -- 24 quantiser runs per block become <= 16,
// 24 prefixes 8.
__global__ void __launch_bounds__(256, 2) k_dual_quant_reg(Params p, Workspace ws)
{
    __shared__ double qc_tab[16];
    if (threadIdx.x < 16) qc_tab[threadIdx.x] = QcDiv{}.at((int)threadIdx.x, 16);
    __syncthreads();
    const QcLds qc{(uint32_t)(uintptr_t)(const __attribute__((address_space(3))) double *)qc_tab};
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t b = gid >> 3, rot = (gid >> 1) & 3u, half = gid & 1u;
    if (b >= p.n) return;
    const BlockMeta meta = ws.meta[b];
    if ((meta.flags & 3u) != 2u) return;
    const bool act4 = mode_active(meta, p, 4), act5 = mode_active(meta, p, 5);
    if (!act4 && !act5) return;
    // the rotation's tasks: mode 4 selection 0, mode 4 selection 1, mode 5
    const uint32_t tk0 = 2 * rot, tk1 = 2 * rot + 1, tk2 = 8 + rot;
    const int n0 = 1 << dual_index_bits(kModes[4], (int)half, 0), n1 = 1 << dual_index_bits(kModes[4], (int)half, 1),
              n2 = 1 << dual_index_bits(kModes[5], (int)half, 0);
    const float *tex = ws.tex + (size_t)b * 64;
    const int c0 = kRot[rot][half ? 0 : 1], c1 = kRot[rot][half ? 0 : 2], c2 = kRot[rot][half ? 0 : 3];
    uint32_t px[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
        px[i] = (uint32_t)tex[i * 4 + c0] | ((uint32_t)tex[i * 4 + c1] << 8) | ((uint32_t)tex[i * 4 + c2] << 16);
    double mean[4] = {0, 0, 0, 0}, dir[4];
    const bool spread = quant_prefix<3>(px, SelPrefix{16}, mean, dir);
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
        const int ncl = pass ? 8 : 4;
        const bool w0 = act4 && n0 == ncl, w1 = act4 && n1 == ncl, w2 = act5 && n2 == ncl;
        if (!(w0 || w1 || w2)) continue;
        double qe = 0.;
        uint64_t ti = 0;
        if (spread) {
            int idx[16], hit = 0;
            qe = opt_quant_from<3>(px, SelPrefix{16}, ncl, idx, mean, dir, qc, &hit);
            if (hit) flag_capped(p, ws, b);
#pragma unroll
            for (int k = 0; k < 16; ++k) ti |= (uint64_t)(idx[k] & 15) << (4 * k);
        }
        const size_t base = (size_t)b * kDualTasks;
        if (w0) {
            ws.dqidx[(base + tk0) * 2 + half] = ti;
            ws.dqerr[(base + tk0) * 2 + half] = qe;
        }
        if (w1) {
            ws.dqidx[(base + tk1) * 2 + half] = ti;
            ws.dqerr[(base + tk1) * 2 + half] = qe;
        }
        if (w2) {
            ws.dqidx[(base + tk2) * 2 + half] = ti;
            ws.dqerr[(base + tk2) * 2 + half] = qe;
        }
    }
}

__global__ void __launch_bounds__(256) k_dual_quant(Params p, Workspace ws)
{
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t b = gid / (kDualTasks * 2), r = gid % (kDualTasks * 2);
    if (b >= p.n) return;
    const uint32_t task = r >> 1, half = r & 1;
    int mode, rot, sel;
    dual_task(task, mode, rot, sel);
    const BlockMeta meta = ws.meta[b];
    if (!mode_active(meta, p, mode) || (meta.flags & 3u)) return;
    const ModeInfo &mi = kModes[mode];
    const float *tex = ws.tex + (size_t)b * 64;
    const int ncl = 1 << dual_index_bits(mi, (int)half, sel);
    double blk[16][4];
    for (int i = 0; i < 16; ++i) {
        for (int j = 0; j < 3; ++j) blk[i][j] = (double)tex[i * 4 + kRot[rot][half ? 0 : j + 1]];
        blk[i][3] = 0.0;
    }
    int idx[16];
    const double qe = opt_quant(blk, 16, ncl, idx, 3);
    uint64_t ti = 0;
    for (int k = 0; k < 16; ++k) ti |= (uint64_t)(idx[k] & 15) << (4 * k);
    ws.dqidx[((size_t)b * kDualTasks + task) * 2 + half] = ti;
    ws.dqerr[((size_t)b * kDualTasks + task) * 2 + half] = qe;
}

// K3t (performance < 1): optQuantTrace_d for both halves of the dual-index
// candidates of blocks whose range exceeds 255 * performance
// (CompressDualIndexBlock :1103-1154); overwrites the optQuantAnD_d results.
__global__ void __launch_bounds__(64) k_dual_quant_trace(Params p, Workspace ws)
{
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t r = gid / p.n, b = gid % p.n;
    if (r >= kDualTasks * 2) return;
    const uint32_t task = r >> 1, half = r & 1;
    int mode, rot, sel;
    dual_task(task, mode, rot, sel);
    const BlockMeta meta = ws.meta[b];
    if (!mode_active(meta, p, mode) || !(meta.max_range > p.quant_thr)) return;
    const ModeInfo &mi = kModes[mode];
    const float *tex = ws.tex + (size_t)b * 64;
    const int ncl = 1 << dual_index_bits(mi, (int)half, sel);
    double blk[16][4];
    for (int i = 0; i < 16; ++i) {
        for (int j = 0; j < 3; ++j) blk[i][j] = (double)tex[i * 4 + kRot[rot][half ? 0 : j + 1]];
        blk[i][3] = 0.0;
    }
    int idx[16];
    const double qe = opt_quant_trace(blk, 16, ncl, idx, 3, p.trace);
    uint64_t ti = 0;
    for (int k = 0; k < 16; ++k) ti |= (uint64_t)(idx[k] & 15) << (4 * k);
    ws.dqidx[((size_t)b * kDualTasks + task) * 2 + half] = ti;
    ws.dqerr[((size_t)b * kDualTasks + task) * 2 + half] = qe;
}

// K3b (waves): shakers of one half of a dual-index candidate
// (CompressDualIndexBlock :1158-1254); integral blocks
template <bool FAST>
__device__ __forceinline__ bool dual_problem(const Params &p, const Workspace &ws, const SpEntry *__restrict__ sp,
                                             uint32_t wid)
{
    const uint32_t b = wid / (kDualTasks * 2), r = wid % (kDualTasks * 2);
    if (b >= p.n) return true;
    const uint32_t task = r >> 1, half = r & 1;
    const int mode = task < 8 ? 4 : 5;
    const int rot = task < 8 ? (int)(task >> 1) : (int)(task - 8);
    const int sel = task < 8 ? (int)(task & 1) : 0;
    const int ln = wv::lane();
    // loads issued before any is waited for (as in k_shake_wave)
    const BlockMeta meta = ws.meta[b];
    const uint32_t pxl = ln < 16 ? ws.px[(size_t)b * 16 + ln] : 0u;   // lane t < 16: texel t, packed
    const uint64_t qi = ws.dqidx[((size_t)b * kDualTasks + task) * 2 + half];
    if (!mode_active(meta, p, mode) || (meta.flags & 3u) != 2u) return true;
    if (!dual_shaken(p, ws, b, (int)task)) {   // not shaken: never selected
        if (ln == 0) ws.dual[(size_t)b * kDualTasks + task].err[half] = 1.7976931348623157e308;
        return true;
    }
    const int shake = dual_shake_size(p);
    const ModeInfo &mi = kModes[mode];
    unsigned px = 0;
#pragma unroll
    for (int j = 0; j < 3; ++j) px |= ((pxl >> (8 * kRot[rot][half ? 0 : j + 1])) & 255u) << (8 * j);
    wv::Texels T;
    wv::make_texels(T, px, 16, 3);
    int idx = T.live ? (int)((qi >> (4 * ln)) & 15u) : 0;
    const int ib = dual_index_bits(mi, (int)half, sel);
    const int last = (1 << ib) - 1;
    const int cb = half ? mi.scalar_bits : mi.vector_bits / 3;
    const int bits[4] = {cb, cb, cb, half ? 6 * cb : 2 * 3 * cb};
    int epo[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    const bool corners_too = !(meta.max_range > p.shake_thr);
    wv::Round0 none;
    none.valid = false;
    double e;
    bool defer = false;
    if (last == 3) {
        if (corners_too) wv::corners<4, FAST>(sp, T, idx, epo, last, bits, PAR_CART, none, defer);   // Q9: error ignored
        if (FAST && defer) return false;
        e = wv::window<4, 3, FAST>(sp, T, idx, epo, shake, last, bits[3], none, defer);
    } else {
        if (corners_too) wv::corners<8, FAST>(sp, T, idx, epo, last, bits, PAR_CART, none, defer);
        if (FAST && defer) return false;
        e = wv::window<8, 3, FAST>(sp, T, idx, epo, shake, last, bits[3], none, defer);
    }
    if (FAST && defer) return false;
    unsigned long long ti = T.live ? (unsigned long long)(idx & 15) << (4 * ln) : 0ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ti |= __shfl_xor(ti, o);
    if (ln == 0) {
        DualResult &res = ws.dual[(size_t)b * kDualTasks + task];
        res.err[half] = e;
        res.idx[half] = ti;
        for (int k = 0; k < 4; ++k) {
            res.ep[half][0][k] = (uint8_t)epo[0][k];
            res.ep[half][1][k] = (uint8_t)epo[1][k];
        }
    }
    return true;
}

__global__ void __launch_bounds__(256, 8) k_dual_wave(Params p, Workspace ws, const SpEntry *__restrict__ sp)
{
    // wave-uniform by construction; readfirstlane lets the compiler see it (scalar loads and branches)
    const uint32_t wid = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    if (!dual_problem<true>(p, ws, sp, wid)) defer_push(p, ws, 3, wid);
}

__global__ void __launch_bounds__(256, 4) k_dual_wave_slow(Params p, Workspace ws, const SpEntry *__restrict__ sp)
{
    const uint32_t w0 = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(ws.defer_cnt[3]);
    const uint32_t *list = ws.defer + (size_t)defer_off(3) * p.n;
    for (uint32_t i = w0; i < cnt; i += nw) dual_problem<false>(p, ws, sp, __builtin_amdgcn_readfirstlane(list[i]));
}

// K3 (f64 lanes): dual-index candidates of blocks with fractional texels
__global__ void __launch_bounds__(256) k_dual(Params p, Workspace ws, const SpEntry *__restrict__ sp)
{
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t b = gid / kDualTasks, task = gid % kDualTasks;
    if (b >= p.n) return;
    const int mode = task < 8 ? 4 : 5;
    const int rot = task < 8 ? (int)(task >> 1) : (int)(task - 8);
    const int sel = task < 8 ? (int)(task & 1) : 0;
    const BlockMeta meta = ws.meta[b];
    if (!mode_active(meta, p, mode) || (meta.flags & 3u)) return;
    if (!dual_shaken(p, ws, b, (int)task)) {   // not shaken: never selected
        ws.dual[(size_t)b * kDualTasks + task].err[0] = 1.7976931348623157e308;
        ws.dual[(size_t)b * kDualTasks + task].err[1] = 1.7976931348623157e308;
        return;
    }
    const ModeInfo &mi = kModes[mode];
    const float *tex = ws.tex + (size_t)b * 64;
    double cb[16][4], ab[16][4];
    for (int i = 0; i < 16; ++i) {
        for (int j = 0; j < 3; ++j) {
            cb[i][j] = (double)tex[i * 4 + kRot[rot][j + 1]];
            ab[i][j] = (double)tex[i * 4 + kRot[rot][0]];
        }
        cb[i][3] = ab[i][3] = 0.0;
    }
    int idx[2][16];
    for (int h = 0; h < 2; ++h) {
        const uint64_t qi = ws.dqidx[((size_t)b * kDualTasks + task) * 2 + h];
        for (int k = 0; k < 16; ++k) idx[h][k] = (int)((qi >> (4 * k)) & 15u);
    }
    const int shake = dual_shake_size(p);
    const int cbits = mi.vector_bits / 3, abits = mi.scalar_bits;
    const int bits0[4] = {cbits, cbits, cbits, 2 * 3 * cbits};
    const int bits1[4] = {abits, abits, abits, 6 * abits};
    const int last0 = (1 << dual_index_bits(mi, 0, sel)) - 1, last1 = (1 << dual_index_bits(mi, 1, sel)) - 1;
    int epo[2][2][4] = {{{0, 0, 0, 0}, {0, 0, 0, 0}}, {{0, 0, 0, 0}, {0, 0, 0, 0}}};
    const bool corners_too = !(meta.max_range > p.shake_thr);
    if (corners_too) shake_corners<double>(sp, cb, &cb[0][0], 16, idx[0], epo[0], last0, bits0, PAR_CART);   // Q9
    const double ec = shake_window<double>(sp, cb, &cb[0][0], 16, idx[0], epo[0], shake, last0, bits0[3], 3);
    if (corners_too) shake_corners<double>(sp, ab, &ab[0][0], 16, idx[1], epo[1], last1, bits1, PAR_CART);
    const double ea = shake_window<double>(sp, ab, &ab[0][0], 16, idx[1], epo[1], shake, last1, bits1[3], 3);
    DualResult &res = ws.dual[(size_t)b * kDualTasks + task];
    res.err[0] = ec;
    res.err[1] = ea;
    for (int h = 0; h < 2; ++h) {
        uint64_t ti = 0;
        for (int k = 0; k < 16; ++k) ti |= (uint64_t)(idx[h][k] & 15) << (4 * k);
        res.idx[h] = ti;
        for (int k = 0; k < 4; ++k) {
            res.ep[h][0][k] = (uint8_t)epo[h][0][k];
            res.ep[h][1][k] = (uint8_t)epo[h][1][k];
        }
    }
}

// K4: mode selection in the reference's visiting order (CompressBlock :1400-1447)
// Mode visit order positions [k0, k1) of CompressBlock's loop; `resume`
// continues from the state an earlier stage stored, k1 == 8 writes the block.
// k_select's per-mode steps.  A dual-index mode's candidate t (mode 4: 8
// rotation x selector tasks, mode 5: 4 rotations) and its score, false when the
// candidate was not shaken (skipped by the choice)
__device__ __forceinline__ bool select_dual_score(const Workspace &ws, uint32_t b, int m, int t, double &v)
{
    const int t0 = m == 4 ? 0 : 8;
    const DualResult &dr = ws.dual[(size_t)b * kDualTasks + t0 + t];
    if (dr.err[0] == 1.7976931348623157e308) return false;   // candidate not shaken
    v = 0;
    v += dr.err[0];
    v += dr.err[1] / 3.;
    return true;
}

// a single-index mode's rank r: its subsets' errors summed in subset order
__device__ __forceinline__ double select_single_score(const Workspace &ws, uint32_t b, int m, int r)
{
    const int slot = m <= 3 ? m : (m == 6 ? 4 : 5);
    const int ns = kModes[m].subsets;
    const ShakeResult *shk = ws.shk + ((size_t)b * kShakeSlots + slot) * kShakeRanks;
    double v = 0;
    for (int s = 0; s < ns; ++s) v += shake_ref(shk, r, s).err[shake_sub(shk, r, s)];
    return v;
}

// the block words of mode m's chosen candidate bi
__device__ __forceinline__ void select_pack(const Workspace &ws, uint32_t b, int m, int bi, uint32_t w[4])
{
    if (m == 4 || m == 5) {
        const int t0 = m == 4 ? 0 : 8;
        const DualResult &dr = ws.dual[(size_t)b * kDualTasks + t0 + bi];
        int ep[2][2][4], idx[2][16];
        for (int h = 0; h < 2; ++h) {
            for (int q = 0; q < 4; ++q) {
                ep[h][0][q] = dr.ep[h][0][q];
                ep[h][1][q] = dr.ep[h][1][q];
            }
            for (int q = 0; q < 16; ++q) idx[h][q] = (int)((dr.idx[h] >> (4 * q)) & 15u);
        }
        const int task = t0 + bi;
        const int rot = task < 8 ? (task >> 1) : (task - 8);
        const int sel = task < 8 ? (task & 1) : 0;
        pack_dual(m, sel, rot, ep, idx, w);
    } else {
        const int slot = m <= 3 ? m : (m == 6 ? 4 : 5);
        const int ns = kModes[m].subsets;
        const ShakeResult *shk = ws.shk + ((size_t)b * kShakeSlots + slot) * kShakeRanks;
        uint8_t ep[3][2][4];
        uint64_t tidx = 0;
        for (int s = 0; s < ns; ++s) {   // repeated subsets: their first occurrence
            const ShakeResult &src = shake_ref(shk, bi, s);
            const int ss = shake_sub(shk, bi, s);
            tidx |= src.idx[ss];
            for (int k = 0; k < 2; ++k)
                for (int c = 0; c < 4; ++c) ep[s][k][c] = src.ep[ss][k][c];
        }
        pack_single(m, (int)shk[bi].part, ep, tidx, w);
    }
}

__global__ void __launch_bounds__(256) k_select(Params p, Workspace ws, uint4 *__restrict__ dst, double *__restrict__ err_out,
                                                int k0, int k1, int resume)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.n) return;
    BlockMeta meta = ws.meta[b];
    const uint32_t out_id = out_block(p, b);
    if (meta.flags & 1u) {
        if (k1 == 8) {
            dst[out_id] = make_uint4(0, 0, 0, 0);
            if (err_out) err_out[out_id] = -1.0;
        }
        return;
    }
    if (p.skip_done && (meta.flags & 4u)) return;   // written by k_bound
    const int order[8] = {6, 4, 3, 1, 2, 0, 7, 5};
    double best = 1.7976931348623157e308, best_d = 1.7976931348623157e308;
    const float *tex = ws.tex + (size_t)b * 64;
    uint32_t bw[4] = {0, 0, 0, 0};
    if (resume) {
        best = ws.best_err[b];
        const uint4 v = ws.best_blk[b];
        bw[0] = v.x;
        bw[1] = v.y;
        bw[2] = v.z;
        bw[3] = v.w;
    }
    for (int k = k0; k < k1; ++k) {
        const int m = order[k];
        if (meta.flags & 4u) break;
        if (!((p.probe ? meta.pvalid : meta.valid) & (1u << m))) continue;
        double be = 1.7976931348623157e308;
        int bi = 0;
        if (m == 4 || m == 5) {
            const int nt = m == 4 ? 8 : 4;
            for (int t = 0; t < nt; ++t) {
                double v;
                if (!select_dual_score(ws, b, m, t, v)) continue;
                if (v < be) {
                    be = v;
                    bi = t;
                }
            }
        } else {
            const int attempts = mode_attempts(p, m);
            for (int r = 0; r < attempts; ++r) {
                const double v = select_single_score(ws, b, m, r);
                if (v < be) {
                    be = v;
                    bi = r;
                }
                if (p.err_thr > 0 && be <= p.err_thr) break;   // :837-843
            }
        }
        const double e = be;
        uint32_t w[4];
        select_pack(ws, b, m, bi, w);
        if (p.decode_select) {
            const double d = decoded_sse(w, tex);
            if (d < best_d) {
                best_d = d;
                best = e;
                for (int q = 0; q < 4; ++q) bw[q] = w[q];
            }
        } else if (e < best) {
            best = e;
            for (int q = 0; q < 4; ++q) bw[q] = w[q];
        }
        if (p.err_thr > 0 && best <= p.err_thr) {   // CompressBlock :1440-1446
            meta.flags |= 4u;
            break;
        }
    }
    if (k1 < 8) {
        ws.best_err[b] = best;
        ws.best_blk[b] = make_uint4(bw[0], bw[1], bw[2], bw[3]);
        ws.meta[b].flags = meta.flags;
        return;
    }
    dst[out_id] = make_uint4(bw[0], bw[1], bw[2], bw[3]);
    if (err_out) err_out[out_id] = best;
}

// k_select for small calls (the block-level entry points): one wave per block.
// Lane 8 k + c scores candidate c of the k-th mode in selection order -- the
// serial kernel's dependent global loads, ~85 us for one block, issued at once --
// and lane 0 replays k_select's choice over the scores from LDS (the same
// comparisons in the same order), then packs only the chosen mode's block.
// Not for the decode-aware choice (bounded-exit probes), which packs every mode.
__global__ void __launch_bounds__(64) k_select_wave(Params p, Workspace ws, uint4 *__restrict__ dst,
                                                    double *__restrict__ err_out, int k0, int k1, int resume)
{
    __shared__ double score[64];
    const uint32_t b = blockIdx.x;
    if (b >= p.n) return;
    const int L = (int)threadIdx.x;
    BlockMeta meta = ws.meta[b];
    const uint32_t out_id = out_block(p, b);
    if (meta.flags & 1u) {
        if (k1 == 8 && L == 0) {
            dst[out_id] = make_uint4(0, 0, 0, 0);
            if (err_out) err_out[out_id] = -1.0;
        }
        return;
    }
    if (p.skip_done && (meta.flags & 4u)) return;   // written by k_bound
    const int order[8] = {6, 4, 3, 1, 2, 0, 7, 5};
    bool has = false;
    {
        const int k = L >> 3, c = L & 7, m = order[k];
        double v = 0;
        if (k >= k0 && k < k1 && ((p.probe ? meta.pvalid : meta.valid) & (1u << m))) {
            if (m == 4 || m == 5)
                has = c < (m == 4 ? 8 : 4) && select_dual_score(ws, b, m, c, v);
            else if (c < mode_attempts(p, m)) {
                v = select_single_score(ws, b, m, c);
                has = true;
            }
        }
        score[L] = v;
    }
    const uint64_t present = __ballot(has);
    __syncthreads();
    if (L != 0) return;
    double best = 1.7976931348623157e308;
    uint32_t bw[4] = {0, 0, 0, 0};
    if (resume) {
        best = ws.best_err[b];
        const uint4 v = ws.best_blk[b];
        bw[0] = v.x;
        bw[1] = v.y;
        bw[2] = v.z;
        bw[3] = v.w;
    }
    int win_m = -1, win_bi = 0;
    for (int k = k0; k < k1; ++k) {
        const int m = order[k];
        if (meta.flags & 4u) break;
        if (!((p.probe ? meta.pvalid : meta.valid) & (1u << m))) continue;
        double be = 1.7976931348623157e308;
        int bi = 0;
        if (m == 4 || m == 5) {
            const int nt = m == 4 ? 8 : 4;
            for (int t = 0; t < nt; ++t) {
                if (!((present >> (8 * k + t)) & 1u)) continue;   // not shaken
                const double v = score[8 * k + t];
                if (v < be) {
                    be = v;
                    bi = t;
                }
            }
        } else {
            const int attempts = mode_attempts(p, m);
            for (int r = 0; r < attempts; ++r) {
                const double v = score[8 * k + r];
                if (v < be) {
                    be = v;
                    bi = r;
                }
                if (p.err_thr > 0 && be <= p.err_thr) break;   // :837-843
            }
        }
        if (be < best) {
            best = be;
            win_m = m;
            win_bi = bi;
        }
        if (p.err_thr > 0 && best <= p.err_thr) {   // CompressBlock :1440-1446
            meta.flags |= 4u;
            break;
        }
    }
    if (win_m >= 0) select_pack(ws, b, win_m, win_bi, bw);
    if (k1 < 8) {
        ws.best_err[b] = best;
        ws.best_blk[b] = make_uint4(bw[0], bw[1], bw[2], bw[3]);
        ws.meta[b].flags = meta.flags;
        return;
    }
    dst[out_id] = make_uint4(bw[0], bw[1], bw[2], bw[3]);
    if (err_out) err_out[out_id] = best;
}

// Bounded exit: the probe stage's block (k_select over one mode with the
// decode-aware choice, stored in ws.best_*) is final when its decode is within
// p.bound_sse of the texels.  With the bound at the contract's absolute slack
// (MSE 0.5 = SSE 32) such a block meets MSE <= MSE_ref * (1 + 1e-3) + 0.5
// whatever the reference's own block is; every other block runs the full
// search, so its output is the exact (or pruned) path's.
__global__ void __launch_bounds__(256) k_bound(Params p, Workspace ws, uint4 *__restrict__ dst,
                                               double *__restrict__ err_out)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.n) return;
    const BlockMeta meta = ws.meta[b];
    if (meta.flags & 5u) return;   // unsupported, or already final
    const double e = ws.best_err[b];
    if (!(e < 1.7976931348623157e308)) return;   // no candidate (the probed mode is not legal here)
    const uint4 v = ws.best_blk[b];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    if (!(decoded_sse(w, ws.tex + (size_t)b * 64) <= p.bound_sse)) return;
    const uint32_t o = out_block(p, b);
    dst[o] = v;
    if (err_out) err_out[o] = e;
    ws.meta[b].flags = meta.flags | 4u;
}

// Stream compaction between bounded-exit stages: the output ids of the
// chunk's blocks that no stage has finished yet (flag bit 2 clear) are
// appended to `out` (one atomic per wave; the order of the list does not
// matter, every block writes its own output slot), so that the next stage's
// launches are sized by the survivors instead of carrying a dead wave per
// finished block through every kernel of the full search.
__global__ void __launch_bounds__(256) k_compact(Params p, Workspace ws, uint32_t *__restrict__ out,
                                                 uint32_t *__restrict__ count)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    const bool keep = b < p.n && !(ws.meta[b].flags & 4u);
    const uint64_t m = __ballot(keep);
    if (!m) return;
    const int lane = (int)__lane_id();
    const int leader = __builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, leader);
    if (keep) out[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = out_block(p, b);
}

// A stage skipped for the rest of its chunks (run_chunks: its first chunk
// finished under 1 % of its blocks): every block of the chunk goes on to the
// next stage's list as it is (k_compact's append, every block kept).
__global__ void __launch_bounds__(256) k_pass_on(Params p, uint32_t *__restrict__ out, uint32_t *__restrict__ count)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t m = __ballot(b < p.n);
    if (!m) return;
    const int lane = (int)__lane_id();
    const int leader = __builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, leader);
    if (b < p.n) out[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = out_block(p, b);
}

// ----------------------------------------------------------------- host ---

static void build_sp_table(std::vector<SpEntry> &tab)
{
    // init_ramps, amd_shake.cpp:302-345 (sp_idx / sp_err), with ramp values
    // from the integer identity above
    const int n_entries = 3 * 4 * 256 * 2 * 2 * 16;
    tab.assign(n_entries, SpEntry{-1, 0, 0xffffffffu});
    auto at = [&](int clog, int bits, int v, int o1, int o2, int i) -> SpEntry & {
        return tab[(((((clog - 2) * 4 + (bits - 5)) * 256 + v) * 2 + o1) * 2 + o2) * 16 + i];
    };
    auto expand = [](int bits, int v) { return (v << (8 - bits)) | (v >> (2 * bits - 8)); };
    auto ramp = [&](int clog, int bits, int p1, int p2, int i) {
        const int e1 = expand(bits, p1), e2 = expand(bits, p2), n = (1 << clog) - 1;
        const int num = 2 * i * (e2 - e1) + n, den = 2 * n;
        int q = num / den;
        if (num < 0 && q * den != num) q--;
        return e1 + q;
    };
    for (int clog = 2; clog < 5; ++clog)
        for (int bits = 5; bits < 9; ++bits)
            for (int p1 = 0; p1 < (1 << bits); ++p1)
                for (int p2 = 0; p2 < (1 << bits); ++p2)
                    for (int i = 0; i < (1 << clog); ++i) {
                        SpEntry &e = at(clog, bits, ramp(clog, bits, p1, p2, i), p1 & 1, p2 & 1, i);
                        e.p1 = (int16_t)p1;
                        e.p2 = (int16_t)p2;
                        e.err = 0;
                    }
    for (int clog = 2; clog < 5; ++clog)
        for (int bits = 5; bits < 9; ++bits)
            for (int v = 0; v < 256; ++v)
                for (int o1 = 0; o1 < 2; ++o1)
                    for (int o2 = 0; o2 < 2; ++o2)
                        for (int i = 0; i < (1 << clog); ++i) {
                            SpEntry &e = at(clog, bits, v, o1, o2, i);
                            if (e.p1 >= 0) continue;
                            int k;
                            for (k = 1; k < 256; ++k)
                                if ((v - k >= 0 && at(clog, bits, v - k, o1, o2, i).err == 0) ||
                                    (v + k < 256 && at(clog, bits, v + k, o1, o2, i).err == 0))
                                    break;
                            if (v - k >= 0 && at(clog, bits, v - k, o1, o2, i).err == 0) {
                                e.p1 = at(clog, bits, v - k, o1, o2, i).p1;
                                e.p2 = at(clog, bits, v - k, o1, o2, i).p2;
                            } else if (v + k < 256 && at(clog, bits, v + k, o1, o2, i).err == 0) {
                                e.p1 = at(clog, bits, v + k, o1, o2, i).p1;
                                e.p2 = at(clog, bits, v + k, o1, o2, i).p2;
                            }
                            e.err = (uint32_t)(k * k);
                        }
}

// distinct subset problems of modes 0-3 (k_quant_sub): 8-cluster ones first
static int build_subset_problems(std::vector<uint32_t> &prob, std::vector<uint32_t> &minpart, std::vector<uint16_t> &tsub)
{
    prob.clear();
    minpart.clear();
    tsub.assign(208 * 3, 0xFFFF);
    auto mask_of = [](uint32_t shape, int j) {
        uint32_t m = 0;
        for (int t = 0; t < 16; ++t) m |= (((shape >> (2 * t)) & 3u) == (uint32_t)j ? 1u : 0u) << t;
        return m;
    };
    for (int pass = 0; pass < 2; ++pass)   // 8 clusters (modes 0, 1), then 4 (modes 2, 3)
        for (int task = 0; task < 208; ++task) {
            const int mode = task < 16 ? 0 : task < 80 ? 1 : task < 144 ? 2 : 3;
            const int part = task < 16 ? task : task < 80 ? task - 16 : task < 144 ? task - 80 : task - 144;
            const int clog = (mode <= 1) ? 3 : 2;
            if ((clog == 3) != (pass == 0)) continue;
            const int subsets = (mode == 0 || mode == 2) ? 3 : 2;
            const uint32_t shape = subsets == 3 ? kBc7Shape3[part] : kBc7Shape2[part];
            for (int j = 0; j < subsets; ++j) {
                const uint32_t key = mask_of(shape, j) | (uint32_t)clog << 16;
                size_t u = 0;
                while (u < prob.size() && prob[u] != key) ++u;
                if (u == prob.size()) {
                    prob.push_back(key);
                    minpart.push_back(0xFFFFFFFFu);
                }
                const uint32_t cur = (minpart[u] >> (8 * mode)) & 0xFFu;
                if ((uint32_t)part < cur)
                    minpart[u] = (minpart[u] & ~(0xFFu << (8 * mode))) | ((uint32_t)part << (8 * mode));
                tsub[task * 3 + j] = (uint16_t)u;
            }
        }
    return (int)prob.size();
}
// the problems paired by mask (k_quant_sub's grid x)
static int build_subset_masks(const std::vector<uint32_t> &prob, std::vector<uint32_t> &pairs)
{
    pairs.clear();
    std::vector<uint32_t> masks;
    for (size_t u = 0; u < prob.size(); ++u) {
        const uint32_t mask = prob[u] & 0xFFFFu;
        const bool eight = (prob[u] >> 16) == 3u;
        size_t i = 0;
        while (i < masks.size() && masks[i] != mask) ++i;
        if (i == masks.size()) {
            masks.push_back(mask);
            pairs.push_back(0xFFFFFFFFu);
        }
        pairs[i] = eight ? (pairs[i] & 0xFFFF0000u) | (uint32_t)u : (pairs[i] & 0xFFFFu) | ((uint32_t)u << 16);
    }
    return (int)pairs.size();
}
static int g_nu = 0, g_nm = 0;

// traceBuilder (amd_bc7_3dquant_vpc.cpp:1557-1712) for ne entries and nc
// clusters, appended to kc/d.  Seven nested loops (one per delimiter, each
// running its positions in the direction given by the parity of its start:
// the reference's DIG macro; a level past nc - 2 runs once) drive a body
// that moves every delimiter one step towards its target position, keeping
// per-cluster counts h (a move that would empty a cluster below zero or put
// every entry in one cluster is retried after the others), and records each
// move.  A jump of more than one position ends the build with no steps, as
// the reference's early return leaves its count at zero.
struct TraceBuild {
    int ne, nc, n, j[7], k[7], h[8], q, q2, cd;
    std::vector<uint32_t> *kc;
    std::vector<double> *d;
    size_t start;
};

static bool trace_body(TraceBuild &b)
{
    bool rescan;
    long guard = 0;
    do {
        rescan = false;
        for (int p = 0; p < b.nc - 1; ++p) {
            const int dj = b.j[p] - b.k[p];
            if (dj < -1 || dj > 1) return false;
            if (!dj) continue;
            const int entry = dj > 0 ? b.k[p] - p : b.j[p] - p;
            const int from = dj > 0 ? p + 1 : p, to = dj > 0 ? p : p + 1;
            if (b.h[from] - 1 < 0 || b.h[to] + 1 >= b.ne) {
                rescan = true;
                continue;
            }
            --b.h[from];
            ++b.h[to];
            b.q2 += dj > 0 ? 1 - 2 * from : 2 * from + 1;
            b.q += dj > 0 ? -1 : 1;
            b.cd = (b.cd | (1 << b.k[p])) & ~(1 << b.j[p]);
            b.kc->push_back((uint32_t)(dj > 0 ? 2 * entry + 1 : 2 * entry) | ((uint32_t)b.cd & 0x7FFFFFFu) << 5);
            b.d->push_back(1. / ((double)b.q2 - (double)b.q * (double)b.q / (double)b.ne));
            b.k[p] = b.j[p];
        }
    } while (rescan && ++guard < 1000000);
    return true;
}

static bool trace_levels(TraceBuild &b, int p, int jin)
{
    const bool used = b.nc >= p + 2;
    for (int i = jin; i < b.n || !used; ++i) {
        b.j[p] = ((jin & 1) == (p & 1)) ? i : b.n - 1 - (i - jin);
        if (!(p < 6 ? trace_levels(b, p + 1, b.j[p] + 1) : trace_body(b))) return false;
        if (!used) break;
    }
    return true;
}

static uint32_t build_trace(int ne, int nc, std::vector<uint32_t> &kc, std::vector<double> &d)
{
    if (nc == 1) return 0;
    TraceBuild b{};
    b.ne = ne, b.nc = nc, b.n = ne + nc - 2;
    for (int p = 0; p < 7; ++p) b.k[p] = p;
    b.h[nc - 1] = ne;
    b.q = ne * (nc - 1);
    b.q2 = ne * (nc - 1) * (nc - 1);
    b.cd = -(1 << (nc - 1));
    b.kc = &kc, b.d = &d;
    const size_t start = kc.size();
    if (!trace_levels(b, 0, 0)) {
        kc.resize(start);
        d.resize(start);
        return 0;
    }
    return (uint32_t)(kc.size() - start);
}

// Per-device state: the single-point table, and two chunk workspaces with two
// internal streams, so that consecutive chunks run concurrently (one chunk's
// quantiser beside the other's shakers, and each launch's tail beside the
// other stream's work) -- chunks are independent, each stays in order on its
// own stream.
// internal streams ("lanes"), each with its own workspace set: consecutive
// chunks go round-robin over them (GIC_BC7_LANES, default 3: 8K exact 4.28 -> 4.21 s
// against 2 lanes, 4 lanes 4.30 s; profiles/r05f_bc7_lanes_ab.txt)
constexpr int kMaxLanes = 4;

struct DeviceState {
    int device = -1;
    SpEntry *sp = nullptr;
    void *ws_mem[kMaxLanes] = {};
    uint32_t ws_blocks[kMaxLanes] = {};
    Workspace ws[kMaxLanes]{};
    hipStream_t lane[kMaxLanes] = {};
    hipEvent_t ev_fork = nullptr, ev_join[kMaxLanes] = {};
    TraceTab trace{nullptr, nullptr};   // optQuantTrace_d tables, built on first use (performance < 1)
    // bounded exit: ping-pong survivor lists (output block ids) and per-stage counters
    uint32_t *list[2] = {nullptr, nullptr};
    uint32_t list_cap = 0;
    uint32_t *count = nullptr;   // [4]
    // H4 re-run list (output ids of capped blocks) and its count
    uint32_t *h4_list = nullptr;
    uint32_t h4_cap = 0;
    uint32_t *h4_cnt = nullptr;
    unsigned long long nonterm_seen = 0;   // g_nonterm at the end of the last call
    // the call's two counters (H4 marks, g_nonterm) copied by one kernel into
    // mapped pinned memory the host reads after its final synchronisation --
    // two synchronous device-to-host copies were ~50 us of a one-block call
    volatile unsigned long long *h_cnt = nullptr;
    unsigned long long *d_cnt = nullptr;
};

__global__ void k_counters(const uint32_t *__restrict__ h4, unsigned long long *__restrict__ out)
{
    out[0] = *h4;
    out[1] = g_nonterm;
}

// Caller holds its device's lock.  Lanes are drained at the end of every call, so
// the list can be replaced here.
static hipError_t get_h4(DeviceState &st, uint32_t total)
{
    hipError_t e = hipSuccess;
    if (!st.h4_cnt) {
        e = hipMalloc(&st.h4_cnt, sizeof(uint32_t));
        if (e != hipSuccess) return e;
    }
    if (!st.h_cnt) {
        void *h = nullptr;
        e = hipHostMalloc(&h, 2 * sizeof(unsigned long long), hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess) return e;
        void *d = nullptr;
        e = hipHostGetDevicePointer(&d, h, 0);
        if (e != hipSuccess) {
            (void)hipHostFree(h);
            return e;
        }
        st.h_cnt = (volatile unsigned long long *)h;
        st.d_cnt = (unsigned long long *)d;
    }
    const uint32_t want = total < (1u << 20) ? total : (1u << 20);   // more marked blocks: re-run the whole call
    if (st.h4_cap >= want) return hipSuccess;
    (void)hipFree(st.h4_list);
    st.h4_list = nullptr;
    st.h4_cap = 0;
    e = hipMalloc(&st.h4_list, (size_t)want * sizeof(uint32_t));
    if (e != hipSuccess) return e;
    st.h4_cap = want;
    return hipSuccess;
}

// Caller holds its device's lock.  The lists are replaced only after both lanes
// drained (earlier calls may still read them).
static hipError_t get_lists(DeviceState &st, uint32_t total)
{
    hipError_t e = hipSuccess;
    if (!st.count) {
        e = hipMalloc(&st.count, 8 * sizeof(uint32_t));   // one survivor counter per stage
        if (e != hipSuccess) return e;
    }
    if (st.list_cap >= total) return hipSuccess;
    for (int k = 0; k < kMaxLanes; ++k) {
        if (st.lane[k]) e = hipStreamSynchronize(st.lane[k]);
        if (e != hipSuccess) return e;
    }
    for (int k = 0; k < 2; ++k) {
        (void)hipFree(st.list[k]);
        st.list[k] = nullptr;
    }
    st.list_cap = 0;
    for (int k = 0; k < 2; ++k) {
        e = hipMalloc(&st.list[k], (size_t)total * sizeof(uint32_t));
        if (e != hipSuccess) return e;
    }
    st.list_cap = total;
    return hipSuccess;
}

// Caller holds its device's lock.
static hipError_t get_trace(DeviceState &st)
{
    if (st.trace.kc) return hipSuccess;
    std::vector<uint32_t> kc;
    std::vector<double> d;
    uint32_t off[8][16], cnt[8][16];
    for (int nc = 1; nc <= 8; ++nc)
        for (int ne = 1; ne <= 16; ++ne) {
            off[nc - 1][ne - 1] = (uint32_t)kc.size();
            cnt[nc - 1][ne - 1] = build_trace(ne, nc, kc, d);
        }
    uint32_t *dkc = nullptr;
    double *dd = nullptr;
    hipError_t e = hipMalloc(&dkc, kc.size() * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&dd, d.size() * sizeof(double));
    if (e == hipSuccess) e = hipMemcpy(dkc, kc.data(), kc.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dd, d.data(), d.size() * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(dTraceOff), off, sizeof(off));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(dTraceCnt), cnt, sizeof(cnt));
    if (e != hipSuccess) {
        (void)hipFree(dkc);
        (void)hipFree(dd);
        return e;
    }
    st.trace.kc = dkc;
    st.trace.d = dd;
    return hipSuccess;
}

// One lock per device: a call holds its device's lock while it enqueues its
// passes (and, for the H4 decision, until they complete), so calls on one
// device are serialised while devices driven from different host threads
// (gic_encode_multi) run concurrently.
static std::mutex g_dev_lock[64];
static DeviceState g_states[64];

static hipError_t current_device(int &dev)
{
    const hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    return (dev < 0 || dev >= 64) ? hipErrorInvalidDevice : hipSuccess;
}

// the host-built tables shared by every device (built once)
struct HostTables {
    std::vector<SpEntry> sp;
    std::vector<uint32_t> prob, minpart, pairs;
    std::vector<uint16_t> tsub;
    int nu = 0, nm = 0;
};
static const HostTables &host_tables()
{
    static HostTables t;
    static std::once_flag once;
    std::call_once(once, [] {
        build_sp_table(t.sp);
        t.nu = build_subset_problems(t.prob, t.minpart, t.tsub);
        t.nm = build_subset_masks(t.prob, t.pairs);
        g_nu = t.nu;
        g_nm = t.nm;
    });
    return t;
}

static size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

// Caller holds its device's lock.  Tables are published (st.sp set) only after
// every upload succeeded; a workspace is reallocated only after its lane has
// drained, since earlier calls may still be using it.
static hipError_t get_state(uint32_t chunk, int nsets, DeviceState *&out)
{
    int dev = 0;
    hipError_t e = current_device(dev);
    if (e != hipSuccess) return e;
    DeviceState &st = g_states[dev];
    if (!st.sp) {
        const HostTables &ht = host_tables();
        const std::vector<SpEntry> &tab = ht.sp;
        SpEntry *sp = nullptr;
        e = hipMalloc(&sp, tab.size() * sizeof(SpEntry));
        if (e != hipSuccess) return e;
        e = hipMemcpy(sp, tab.data(), tab.size() * sizeof(SpEntry), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(dShape2), kBc7Shape2, sizeof(kBc7Shape2));
        if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(dShape3), kBc7Shape3, sizeof(kBc7Shape3));
        if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(dAnchor2), kBc7Anchor2, sizeof(kBc7Anchor2));
        if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(dAnchor3a), kBc7Anchor3a, sizeof(kBc7Anchor3a));
        if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(dAnchor3b), kBc7Anchor3b, sizeof(kBc7Anchor3b));
        if (e == hipSuccess && ht.nu > kUMax) e = hipErrorInvalidValue;
        if (e == hipSuccess)
            e = hipMemcpyToSymbol(HIP_SYMBOL(dUProb), ht.prob.data(), ht.prob.size() * sizeof(uint32_t));
        if (e == hipSuccess)
            e = hipMemcpyToSymbol(HIP_SYMBOL(dUMinPart), ht.minpart.data(), ht.minpart.size() * sizeof(uint32_t));
        if (e == hipSuccess)
            e = hipMemcpyToSymbol(HIP_SYMBOL(dTaskSub), ht.tsub.data(), ht.tsub.size() * sizeof(uint16_t));
        if (e == hipSuccess)
            e = hipMemcpyToSymbol(HIP_SYMBOL(dUMask), ht.pairs.data(), ht.pairs.size() * sizeof(uint32_t));
        if (e != hipSuccess) {
            (void)hipFree(sp);
            return e;
        }
        st.device = dev;
        st.sp = sp;
    }
    if (!st.lane[0]) {
        for (int k = 0; k < kMaxLanes; ++k) {
            e = hipStreamCreateWithFlags(&st.lane[k], hipStreamNonBlocking);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&st.ev_join[k], hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
        e = hipEventCreateWithFlags(&st.ev_fork, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    for (int k = 0; k < nsets; ++k) {
        if (st.ws_blocks[k] >= chunk) continue;
        if (st.ws_mem[k]) {
            e = hipStreamSynchronize(st.lane[k]);   // earlier calls' passes on this workspace
            if (e != hipSuccess) return e;
            (void)hipFree(st.ws_mem[k]);
        }
        st.ws_mem[k] = nullptr;
        st.ws_blocks[k] = 0;
        const size_t n = chunk;
        const size_t sz = align_up(n * 64 * sizeof(float)) + align_up(n * sizeof(BlockMeta)) +
                          align_up(n * kQuantTasks * sizeof(double)) + align_up(n * kQuantTasks * sizeof(uint64_t)) +
                          align_up(n * kShakeSlots * kShakeRanks * sizeof(ShakeResult)) +
                          align_up(n * kShakeSlots * kShakeRanks) +
                          align_up(n * kDualTasks * sizeof(DualResult)) + align_up(n * kDualTasks * 2 * sizeof(uint64_t)) +
                          align_up(n * kDualTasks * 2 * sizeof(double)) + align_up(n * sizeof(double)) +
                          align_up(n * sizeof(uint4)) + align_up(n * kUMax * sizeof(double)) +
                          align_up(n * kUMax * sizeof(uint64_t)) +
                          align_up(n * kShakeSlots * kShakeRanks * sizeof(uint64_t)) + align_up(n * 16 * sizeof(uint32_t)) +
                          align_up(n * kDeferPer * sizeof(uint32_t)) + align_up(4 * sizeof(uint32_t));
        e = hipMalloc(&st.ws_mem[k], sz);
        if (e != hipSuccess) return e;
        Workspace &w = st.ws[k];
        char *p = (char *)st.ws_mem[k];
        w.tex = (float *)p;
        p += align_up(n * 64 * sizeof(float));
        w.meta = (BlockMeta *)p;
        p += align_up(n * sizeof(BlockMeta));
        w.qerr = (double *)p;
        p += align_up(n * kQuantTasks * sizeof(double));
        w.qidx = (uint64_t *)p;
        p += align_up(n * kQuantTasks * sizeof(uint64_t));
        w.shk = (ShakeResult *)p;
        p += align_up(n * kShakeSlots * kShakeRanks * sizeof(ShakeResult));
        w.prank = (uint8_t *)p;
        p += align_up(n * kShakeSlots * kShakeRanks);
        w.dual = (DualResult *)p;
        p += align_up(n * kDualTasks * sizeof(DualResult));
        w.dqidx = (uint64_t *)p;
        p += align_up(n * kDualTasks * 2 * sizeof(uint64_t));
        w.dqerr = (double *)p;
        p += align_up(n * kDualTasks * 2 * sizeof(double));
        w.best_err = (double *)p;
        p += align_up(n * sizeof(double));
        w.best_blk = (uint4 *)p;
        p += align_up(n * sizeof(uint4));
        w.uerr = (double *)p;
        p += align_up(n * kUMax * sizeof(double));
        w.uidx = (uint64_t *)p;
        p += align_up(n * kUMax * sizeof(uint64_t));
        w.pqidx = (uint64_t *)p;
        p += align_up(n * kShakeSlots * kShakeRanks * sizeof(uint64_t));
        w.px = (uint32_t *)p;
        p += align_up(n * 16 * sizeof(uint32_t));
        w.defer = (uint32_t *)p;
        p += align_up(n * kDeferPer * sizeof(uint32_t));
        w.defer_cnt = (uint32_t *)p;
        st.ws_blocks[k] = chunk;
    }
    out = &st;
    return hipSuccess;
}

// K1-K3 for the modes of p.stage_mask (kernels return early for inactive work)
// `integral`: every block of the chunk has integral texels in [0, 255] (an
// 8-bit image source: v / 255.0f * 255.0f is exact for every byte), so the
// f64 fallback kernels (k_quant, k_shake, k_dual_quant, k_dual) would only
// read the flags and exit; they are not launched (their 1-wave/SIMD grids
// otherwise wait for whole SIMDs behind the other lane's shakers).
static hipError_t run_modes(const Params &p, const Workspace &ws, const SpEntry *sp, hipStream_t s, bool integral)
{
    const uint32_t wg = 256;
    const uint32_t sm = p.stage_mask;
    const bool single = (sm & 0xCFu) != 0, dual = (sm & 0x30u) != 0;
    // deferred shake problems of this pass (fast wave kernels -> slow ones);
    // the slow kernels' grid: 4 waves per SIMD (their VGPRs allow 4), striding
    // over the lists.  The counters must be zero before the fast kernels
    // append: a failed reset stops the pass.
    const hipError_t me = hipMemsetAsync(ws.defer_cnt, 0, 4 * sizeof(uint32_t), s);
    if (me != hipSuccess) return me;
    const dim3 slow_grid(1024);
    if (single) {
        const uint64_t nq = (uint64_t)p.n * kQuantTasks;
        if (!integral) hipLaunchKernelGGL(k_quant, dim3((uint32_t)((nq + wg - 1) / wg)), dim3(wg), 0, s, p, ws);
        const uint64_t nq3 = (uint64_t)p.n * 208, nq4 = (uint64_t)p.n * 65;
        if (sm & 0x0Fu) {
            hipLaunchKernelGGL(k_quant_sub, dim3((uint32_t)g_nm, (p.n + wg - 1) / wg), dim3(wg), 0, s, p, ws);
            hipLaunchKernelGGL(k_quant_gather, dim3((uint32_t)((nq3 + wg - 1) / wg)), dim3(wg), 0, s, p, ws);
        }
        if ((sm & 0xC0u) == 0x40u && p.probe) {   // the bounded exit's mode-6 probe: first projection only
            hipLaunchKernelGGL(k_quant_probe6, dim3((p.n + wg - 1) / wg), dim3(wg), 0, s, p, ws);
        } else if ((sm & 0xC0u) == 0x40u) {   // mode 6 alone: one lane per block
            hipLaunchKernelGGL(k_quant_reg<4>, dim3((p.n + wg - 1) / wg), dim3(wg), 0, s, p, ws, 208, 1);
        } else if (sm & 0xC0u) {
            hipLaunchKernelGGL(k_quant_reg<4>, dim3((uint32_t)((nq4 + wg - 1) / wg)), dim3(wg), 0, s, p, ws, 208, 65);
        }
        if (p.quant_thr < 255.0 && (sm & 0x8Fu)) {
            const uint64_t nt = (uint64_t)p.n * 272;
            hipLaunchKernelGGL(k_quant_trace, dim3((uint32_t)((nt + 63) / 64)), dim3(64), 0, s, p, ws);
        }
        const uint64_t ns = (uint64_t)p.n * kShakeSlots * kShakeRanks;
        if (!integral) hipLaunchKernelGGL(k_shake, dim3((uint32_t)((ns + wg - 1) / wg)), dim3(wg), 0, s, p, ws, sp);
        if (sm & 0x8Fu) {   // partition ranks of the multi-partition modes (mode 6 has one partition)
            const uint64_t nr = (uint64_t)p.n * kShakeSlots * 64;
            hipLaunchKernelGGL(k_rank, dim3((uint32_t)((nr + wg - 1) / wg)), dim3(wg), 0, s, p, ws);
        }
        if ((sm & 0x03u) && wave_count<8>(p.att)) {
            const uint64_t nw8 = (uint64_t)p.n * wave_count<8>(p.att) * 64;
            hipLaunchKernelGGL(k_shake_wave<8>, dim3((uint32_t)((nw8 + wg - 1) / wg)), dim3(wg), 0, s, p, ws, sp);
        }
        if ((sm & 0x8Cu) && wave_count<4>(p.att)) {
            const uint64_t nw4 = (uint64_t)p.n * wave_count<4>(p.att) * 64;
            hipLaunchKernelGGL(k_shake_wave<4>, dim3((uint32_t)((nw4 + wg - 1) / wg)), dim3(wg), 0, s, p, ws, sp);
        }
        if (sm & 0x40u) {
            const uint64_t nw16 = (uint64_t)p.n * wave_count<16>(p.att) * 64;
            hipLaunchKernelGGL(k_shake_wave<16>, dim3((uint32_t)((nw16 + wg - 1) / wg)), dim3(wg), 0, s, p, ws, sp);
        }
        if ((sm & 0x03u) && wave_count<8>(p.att))
            hipLaunchKernelGGL(k_shake_wave_slow<8>, slow_grid, dim3(wg), 0, s, p, ws, sp);
        if ((sm & 0x8Cu) && wave_count<4>(p.att))
            hipLaunchKernelGGL(k_shake_wave_slow<4>, slow_grid, dim3(wg), 0, s, p, ws, sp);
        if (sm & 0x40u) hipLaunchKernelGGL(k_shake_wave_slow<16>, slow_grid, dim3(wg), 0, s, p, ws, sp);
    }
    if (dual) {
        const uint64_t ndq = (uint64_t)p.n * kDualTasks * 2;
        if (!integral) hipLaunchKernelGGL(k_dual_quant, dim3((uint32_t)((ndq + wg - 1) / wg)), dim3(wg), 0, s, p, ws);
        const uint64_t ndr = (uint64_t)p.n * 8;   // (block, rotation, half)
        hipLaunchKernelGGL(k_dual_quant_reg, dim3((uint32_t)((ndr + wg - 1) / wg)), dim3(wg), 0, s, p, ws);
        if (p.quant_thr < 255.0)
            hipLaunchKernelGGL(k_dual_quant_trace, dim3((uint32_t)((ndq + 63) / 64)), dim3(64), 0, s, p, ws);
        const uint64_t nd = (uint64_t)p.n * kDualTasks;
        if (!integral) hipLaunchKernelGGL(k_dual, dim3((uint32_t)((nd + wg - 1) / wg)), dim3(wg), 0, s, p, ws, sp);
        const uint64_t ndw = (uint64_t)p.n * kDualTasks * 2 * 64;
        hipLaunchKernelGGL(k_dual_wave, dim3((uint32_t)((ndw + wg - 1) / wg)), dim3(wg), 0, s, p, ws, sp);
        hipLaunchKernelGGL(k_dual_wave_slow, slow_grid, dim3(wg), 0, s, p, ws, sp);
    }
    return hipGetLastError();
}

#ifndef GIC_BC7_CHUNK
#define GIC_BC7_CHUNK 65536
#endif
constexpr uint32_t kChunk = GIC_BC7_CHUNK;   // blocks per pipeline pass (~1.1 GB workspace per set at 65536)

// BC7BlockEncoder constructor (amd_bc7_body.hpp:94-149): the quality- and
// performance-derived settings of every pass
static void base_params(const gic_options &o, const DeviceState &st, double perf, Params &p)
{
    p.mode_mask = o.bc7_mode_mask;
    p.colour_restrict = o.colour_restrict;
    p.alpha_restrict = o.alpha_restrict;
    p.force_alpha_one = o.force_alpha_one;
    const double q = o.bc7_quality;
    p.quality = q < 1.0 ? (q > 0.0 ? q : 0.0) : 1.0;
    if (p.quality < 0.5) {
        p.shake_thr = 0.;
        p.err_thr = 256. * (1.0 - ((p.quality * 2.0) / 0.5));
        p.part_search = (1.0 / 16.0) > ((p.quality * 2.0) / 0.5) ? (1.0 / 16.0) : ((p.quality * 2.0) / 0.5);
    } else if (p.quality < 0.7) {
        p.shake_thr = 255 * (p.quality / 10);
        p.err_thr = 256. * (1.0 - (p.quality / 0.5));
        p.part_search = (1.0 / 16.0) > (p.quality / 0.5) ? (1.0 / 16.0) : (p.quality / 0.5);
    } else {
        p.shake_thr = 255 * p.quality;
        p.err_thr = 0;
        p.part_search = 1.0;
    }
    p.quant_thr = 255 * perf;
    p.trace = st.trace;
    p.att = host_attempts(p, o.bc7_shake_ranks);
    p.decode_select = o.bc7_shake_ranks > 0 && !(p.err_thr > 0);
    p.dual_cap = 2 * (int)o.bc7_shake_ranks;
    p.bound_sse = 0.0;
    p.skip_done = 0;
    p.probe = 0;
    p.stage_mask = 0xFFu;
    p.list = nullptr;
    p.first = 0;
    p.n = 0;
    p.h4_list = st.h4_list;
    p.h4_cnt = st.h4_cnt;
    p.h4_cap = st.h4_cap;
    p.general = 0;
}

// H4 report of the calling thread's last BC7 call (gic_last_h4_report)
thread_local uint32_t t_h4_rerun = 0, t_h4_nonterm = 0;
// blocks entering each stage of the calling thread's last BC7 call
// (gic_last_bc7_stages): bounded exit = mode-6 fit, probes 6, 3, 1 and 4, search
thread_local uint32_t t_stage_in[6] = {0, 0, 0, 0, 0, 0};
thread_local int t_nstages = 0;

static hipError_t run_chunks(const Geometry *g, const float *blocks, uint32_t total, const gic_options &o, void *dst,
                             double *err, hipStream_t s)
{
    const uint32_t chunk = total < kChunk ? total : kChunk;
    // GIC_BC7_SINGLE_STREAM=1: every chunk on one lane (per-kernel profiles
    // then attribute time without the two lanes' overlap)
    static const bool single_stream = getenv("GIC_BC7_SINGLE_STREAM") && atoi(getenv("GIC_BC7_SINGLE_STREAM"));
    static const int lanes_env = getenv("GIC_BC7_LANES") ? atoi(getenv("GIC_BC7_LANES")) : 3;
    const int lanes = lanes_env < 1 ? 1 : (lanes_env > kMaxLanes ? kMaxLanes : lanes_env);
    const uint32_t nchunks = (total + chunk - 1) / chunk;
    const int nsets = single_stream ? 1 : (int)(nchunks < (uint32_t)lanes ? nchunks : (uint32_t)lanes);
    // Workspace k is used only on lane k, and a call enqueues all its passes
    // while holding the device lock: concurrent calls (other threads, other
    // caller streams) are serialised in lane order, never interleaved on a
    // workspace.  The caller's stream is joined by fork/join events.
    int dev = 0;
    hipError_t e = current_device(dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(g_dev_lock[dev]);
    DeviceState *st = nullptr;
    e = get_state(chunk, nsets, st);
    if (e != hipSuccess) return e;
    // BC7BlockEncoder ctor: m_performance clamped to [0, 1], m_quantizerRangeThreshold
    // = 255 * m_performance (amd_bc7_body.hpp:109-116)
    const double perf = o.bc7_performance < 1.0 ? (o.bc7_performance > 0.0 ? (double)o.bc7_performance : 0.0) : 1.0;
    if (perf < 1.0) {
        e = get_trace(*st);
        if (e != hipSuccess) return e;
    }
    e = get_h4(*st, total);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(st->h4_cnt, 0, sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    t_h4_rerun = t_h4_nonterm = 0;
    Params base;
    base_params(o, *st, perf, base);
    // err_thr > 0 (quality < 0.25): CompressBlock stops visiting modes once a
    // block's best error is within the threshold, so the modes run one stage
    // at a time in visit order and finished blocks drop out of later stages.
    const bool staged = base.err_thr > 0;
    const bool bounded = o.bc7_mse_bound > 0.f && !staged;
    const int order[8] = {6, 4, 3, 1, 2, 0, 7, 5};
    const uint32_t valid_modes = o.bc7_mode_mask == 0 ? 0xCFu : o.bc7_mode_mask;
    if (bounded) {
        e = get_lists(*st, total);
        if (e != hipSuccess) return e;
        e = hipMemsetAsync(st->count, 0, 8 * sizeof(uint32_t), s);
        if (e != hipSuccess) return e;
    }
    e = hipEventRecord(st->ev_fork, s);   // fork: the lanes start after the caller's prior work
    for (int k = 0; k < nsets && e == hipSuccess; ++k) e = hipStreamWaitEvent(st->lane[k], st->ev_fork, 0);
    if (e != hipSuccess) return e;
    const hipStream_t caller = s;
    const uint32_t wg = 256;
    // Stages: without the bounded exit one (the search); with it the probes
    // (modes 6, 3, then 1 -- visit positions 0, 2, 3 -- each with two
    // partitions shaken and the decode-aware choice; k_bound makes a block
    // final when its probe block decodes within the bound), then the full
    // search over the blocks no probe finished.  Between stages the
    // unfinished blocks are compacted into a list (k_compact) and the next
    // stage runs over that list in dense chunks.  The probes may use mode 6
    // on opaque blocks, which the reference's colour restriction leaves out
    // of its own search: any BC7 block within the bound meets the contract.
    // Stage 0 (-2, before the probes): the direct mode-6 fit (k_fit6).
    int stages[6], nstages = 0;
    if (bounded) {
        if (valid_modes & 0x40u) stages[nstages++] = -2;
        for (int k : {0, 2, 3, 1})   // modes 6, 3, 1, then 4
            if (valid_modes & (1u << order[k])) stages[nstages++] = k;
    }
    stages[nstages++] = -1;   // the search itself
    // the search over one chunk (the modes in one launch sequence, or staged)
    auto search = [&](Params p, const Workspace &ws, hipStream_t s, bool integral) -> hipError_t {
        int resume = 0;
        for (int k = 0; k < (staged ? 8 : 1); ++k) {
            p.stage_mask = staged ? (1u << order[k]) : 0xFFu;
            const bool last = !staged || k == 7;
            const bool skip = staged && !(valid_modes & p.stage_mask);
            if (skip && !last) continue;
            if (!skip) {
                const hipError_t re = run_modes(p, ws, st->sp, s, integral);
                if (re != hipSuccess) return re;
            }
            if (p.n < kSelectWaveBlocks && !p.decode_select)
                hipLaunchKernelGGL(k_select_wave, dim3(p.n), dim3(64), 0, s, p, ws, (uint4 *)dst, err, staged ? k : 0,
                                   staged ? k + 1 : 8, resume);
            else
                hipLaunchKernelGGL(k_select, dim3((p.n + wg - 1) / wg), dim3(wg), 0, s, p, ws, (uint4 *)dst, err,
                                   staged ? k : 0, staged ? k + 1 : 8, resume);
            resume = 1;
        }
        return hipGetLastError();
    };
    const uint32_t *cur = nullptr;
    uint32_t cur_n = total;
    uint32_t ci = 0;
    for (int k = 0; k < 6; ++k) t_stage_in[k] = 0;
    t_nstages = nstages;
    // A probe stage (stage 0 included) whose first chunk finishes under 1 % of
    // its blocks is skipped for the rest of the call: its remaining chunks go
    // on to the next stage untouched (k_pass_on).  On content no probe suits
    // (G2: independent channel noise, 0 % within the bound) the bounded exit
    // then costs what the search does, plus one chunk per probe; which blocks a
    // skipped chunk would have finished only changes which contract-meeting
    // block they get (the search's own).
    for (int si = 0; si < nstages && cur_n; ++si) {
        const int pk = stages[si];
        t_stage_in[si] = cur_n;
        const bool last_stage = si == nstages - 1;
        uint32_t *out = bounded ? st->list[si & 1] : nullptr;
        bool skip_rest = false;
        for (uint32_t first = 0; first < cur_n; first += chunk, ++ci) {
            const Workspace &ws = st->ws[ci % (uint32_t)nsets];
            s = st->lane[ci % (uint32_t)nsets];
            Params p = base;
            p.first = first;
            p.n = (cur_n - first) < chunk ? (cur_n - first) : chunk;
            p.list = cur ? cur + first : nullptr;
            if (!last_stage && first == chunk && cur_n > 2 * chunk) {
                // the first chunk's survivors: its lane is drained for the count
                e = hipStreamSynchronize(st->lane[(ci - 1) % (uint32_t)nsets]);
                uint32_t kept = 0;
                if (e == hipSuccess) e = hipMemcpy(&kept, st->count + si, sizeof(uint32_t), hipMemcpyDeviceToHost);
                if (e != hipSuccess) return e;
                skip_rest = (uint64_t)(chunk - kept) * 100u < (uint64_t)chunk;
            }
            if (skip_rest) {
                hipLaunchKernelGGL(k_pass_on, dim3((p.n + wg - 1) / wg), dim3(wg), 0, s, p, out, st->count + si);
                e = hipGetLastError();
                if (e != hipSuccess) return e;
                continue;
            }
            if (g)
                hipLaunchKernelGGL(k_prep_image, dim3((p.n + wg - 1) / wg), dim3(wg), 0, s, *g, p, ws);
            else
                hipLaunchKernelGGL(k_prep_f32, dim3((p.n + wg - 1) / wg), dim3(wg), 0, s, blocks, p, ws);
            if (pk == -2) {
                Params pp = p;
                pp.bound_sse = 64.0 * (double)o.bc7_mse_bound;
                pp.probe = 1;
                pp.stage_mask = 0x40u;
                hipLaunchKernelGGL(k_quant_probe6, dim3((p.n + wg - 1) / wg), dim3(wg), 0, s, pp, ws);
                hipLaunchKernelGGL(k_fit6, dim3((p.n + wg - 1) / wg), dim3(wg), 0, s, pp, ws, (uint4 *)dst, err);
                hipLaunchKernelGGL(k_compact, dim3((p.n + wg - 1) / wg), dim3(wg), 0, s, pp, ws, out,
                                   st->count + si);
            } else if (pk >= 0) {
                Params pp = p;
                pp.att = host_attempts(pp, 2);
                pp.decode_select = 1;
                pp.dual_cap = 4;
                pp.bound_sse = 64.0 * (double)o.bc7_mse_bound;
                pp.probe = 1;
                pp.stage_mask = 1u << order[pk];
                e = run_modes(pp, ws, st->sp, s, g != nullptr);
                if (e != hipSuccess) return e;
                hipLaunchKernelGGL(k_select, dim3((p.n + wg - 1) / wg), dim3(wg), 0, s, pp, ws, (uint4 *)dst, err,
                                   pk, pk + 1, 0);
                hipLaunchKernelGGL(k_bound, dim3((p.n + wg - 1) / wg), dim3(wg), 0, s, pp, ws, (uint4 *)dst, err);
                hipLaunchKernelGGL(k_compact, dim3((p.n + wg - 1) / wg), dim3(wg), 0, s, pp, ws, out,
                                   st->count + si);
            } else {
                e = search(p, ws, s, g != nullptr);
                if (e != hipSuccess) return e;
            }
            e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        if (!last_stage) {
            // the survivor count sizes the next stage's passes (a host round
            // trip per stage; the lanes are drained anyway)
            for (int k = 0; k < nsets && e == hipSuccess; ++k) e = hipStreamSynchronize(st->lane[k]);
            uint32_t n_next = 0;
            if (e == hipSuccess) e = hipMemcpy(&n_next, st->count + si, sizeof(uint32_t), hipMemcpyDeviceToHost);
            if (e != hipSuccess) return e;
            if (n_next > cur_n) return hipErrorUnknown;   // cannot happen: a stage only removes blocks
            cur = out;
            cur_n = n_next;
        }
    }
    // H4: blocks whose register quantiser stopped at the iteration cap are
    // encoded again through the general kernels (uncapped, cycle-checked
    // quantiser), so their output is the reference's.  Deciding needs the
    // marked count on the host: a BC7 call returns with its work complete.
    // lane 0 waits for the others, copies both counters to the mapped words, and
    // one synchronisation covers the whole call
    for (int k = 1; k < nsets && e == hipSuccess; ++k) {
        e = hipEventRecord(st->ev_join[k], st->lane[k]);
        if (e == hipSuccess) e = hipStreamWaitEvent(st->lane[0], st->ev_join[k], 0);
    }
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_counters, dim3(1), dim3(1), 0, st->lane[0], st->h4_cnt, st->d_cnt);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(st->lane[0]);
    if (e != hipSuccess) return e;
    const uint32_t nh = (uint32_t)st->h_cnt[0];
    unsigned long long nt_end = st->h_cnt[1];
    if (nh > 0) {
        const uint32_t *rl = nh <= st->h4_cap ? st->h4_list : nullptr;   // overflow: the whole call
        const uint32_t rn = rl ? nh : total;
        for (uint32_t first = 0; first < rn; first += chunk) {
            const Workspace &ws = st->ws[0];
            s = st->lane[0];
            Params p = base;
            p.general = 1;
            p.first = first;
            p.n = (rn - first) < chunk ? (rn - first) : chunk;
            p.list = rl ? rl + first : nullptr;
            if (g)
                hipLaunchKernelGGL(k_prep_image, dim3((p.n + wg - 1) / wg), dim3(wg), 0, s, *g, p, ws);
            else
                hipLaunchKernelGGL(k_prep_f32, dim3((p.n + wg - 1) / wg), dim3(wg), 0, s, blocks, p, ws);
            e = search(p, ws, s, false);
            if (e != hipSuccess) return e;
        }
        e = hipStreamSynchronize(st->lane[0]);
        if (e != hipSuccess) return e;
        t_h4_rerun = rn;
        e = hipMemcpyFromSymbol(&nt_end, HIP_SYMBOL(g_nonterm), sizeof(nt_end));   // the re-run's cycles
        if (e != hipSuccess) return e;
    }
    t_h4_nonterm = (uint32_t)(nt_end - st->nonterm_seen);
    st->nonterm_seen = nt_end;
    {   // join: the caller's stream waits for the lanes
        for (int k = 0; k < nsets && e == hipSuccess; ++k) {
            e = hipEventRecord(st->ev_join[k], st->lane[k]);
            if (e == hipSuccess) e = hipStreamWaitEvent(caller, st->ev_join[k], 0);
        }
    }
    return e;
}

}  // namespace bc7

namespace bc7 {
__global__ void __launch_bounds__(256) k_decode(const uint4 *__restrict__ blocks, uint32_t width, uint32_t height,
                                                uint32_t bx_count, uint32_t total, uint8_t *__restrict__ out,
                                                size_t row_pitch)
{
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= total) return;
    const uint32_t by_count = (height + 3) / 4;
    const uint32_t bx = id % bx_count, r = id / bx_count, by = r % by_count, slice = r / by_count;
    const uint4 b = blocks[id];
    const uint32_t w[4] = {b.x, b.y, b.z, b.w};
    uint32_t px[16];
    bc7_decode_block(w, px);
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
}  // namespace bc7

hipError_t launch_bc7_decode(const uint8_t *blocks, uint32_t width, uint32_t height, uint32_t slices, uint8_t *out,
                             size_t row_pitch, hipStream_t s)
{
    {   // the partition / anchor tables live in this library's constant memory
        int dev = 0;
        hipError_t e = bc7::current_device(dev);
        if (e != hipSuccess) return e;
        std::lock_guard<std::mutex> lk(bc7::g_dev_lock[dev]);
        bc7::DeviceState *st = nullptr;
        e = bc7::get_state(0, 0, st);
        if (e != hipSuccess) return e;
    }
    const uint32_t bx = (width + 3) / 4, by = (height + 3) / 4;
    const uint64_t total = (uint64_t)bx * by * slices;
    if (total > 0xffffffffull) return hipErrorInvalidValue;
    const uint32_t wg = 256, grid = (uint32_t)((total + wg - 1) / wg);
    hipLaunchKernelGGL(bc7::k_decode, dim3(grid), dim3(wg), 0, s, (const uint4 *)blocks, width, height, bx,
                       (uint32_t)total, out, row_pitch);
    return hipGetLastError();
}

hipError_t launch_bc7_image(const Geometry &g, const gic_options &o, void *dst, double *err, hipStream_t s)
{
    return bc7::run_chunks(&g, nullptr, g.total, o, dst, err, s);
}

hipError_t launch_bc7_blocks(const float *blocks, uint32_t n, const gic_options &o, void *dst, double *err,
                             hipStream_t s)
{
    return bc7::run_chunks(nullptr, blocks, n, o, dst, err, s);
}

hipError_t bc7_nonterm(unsigned long long *n, int reset)
{
    int dev = 0;
    hipError_t e = bc7::current_device(dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(bc7::g_dev_lock[dev]);
    e = hipMemcpyFromSymbol(n, HIP_SYMBOL(bc7::g_nonterm), sizeof(*n));
    if (e == hipSuccess && reset) {
        const unsigned long long z = 0;
        e = hipMemcpyToSymbol(HIP_SYMBOL(bc7::g_nonterm), &z, sizeof(z));
        if (e == hipSuccess) bc7::g_states[dev].nonterm_seen = 0;
    }
    return e;
}

void bc7_last_stages(uint32_t in[6], int *n)
{
    for (int k = 0; k < 6; ++k) in[k] = bc7::t_stage_in[k];
    *n = bc7::t_nstages;
}

void bc7_last_h4(uint32_t *rerun, uint32_t *nonterm)
{
    if (rerun) *rerun = bc7::t_h4_rerun;
    if (nonterm) *nonterm = bc7::t_h4_nonterm;
}

}  // namespace gic

namespace gic {
hipError_t bc7_iter_cap(int cap, unsigned long long *hits, int reset)
{
    hipError_t e = hipSuccess;
    if (hits) e = hipMemcpyFromSymbol(hits, HIP_SYMBOL(bc7::g_iter_hits), sizeof(*hits));
    if (e == hipSuccess && reset) {
        const unsigned long long z = 0;
        e = hipMemcpyToSymbol(HIP_SYMBOL(bc7::g_iter_hits), &z, sizeof(z));
    }
    if (e == hipSuccess && cap >= 0) e = hipMemcpyToSymbol(HIP_SYMBOL(bc7::g_iter_cap), &cap, sizeof(cap));
    return e;
}
}  // namespace gic

#ifdef GIC_PROFILE
extern "C" int gic_debug_profile(unsigned long long out[32], int reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gic::bc7::wv::g_prof), 32 * sizeof(unsigned long long)) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[32] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(gic::bc7::wv::g_prof), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

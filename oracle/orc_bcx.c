/*
 * orc_bcx.c -- CPU restatement of the reference BC1 / BC4 (BC5) block search.
 *
 * TEST INFRASTRUCTURE ONLY (see bcn_oracle.h).  Restates, for the default
 * options path, src/amd_bcx_body.cpp and src/amd_bcx_helpers.cpp of
 * DeanoC/gfx_imagecompress.  Float/double types and the association order of
 * every non-exact expression follow the reference so results are bit-exact;
 * build with -ffp-contract=off (no FMA contraction, no fast-math).
 *
 * Channel order inside the colour path is the reference's B,G,R
 * (amd_bcx_body.cpp:60-63).
 */
#include "bcn_oracle.h"
#ifdef ORC_STATS
__thread long orc_bcx_stat[4];   /* study counters (tools/bc1_iter_study.c) */
/* study hook: every RampSrchW call's running sums without the early break
 * (tools/bc1_cut_study.c) */
void (*orc_bcx_ramp_hook)(const float run[16], const float perr[16], float maxerr, int ncol, int n);
#endif

#include <float.h>
#include <math.h>
#include <string.h>

enum { CH_B = 0, CH_G = 1, CH_R = 2, CH_A = 3 };

#define BCX_MAX_ERROR 128000.f            /* amd_bcx_body.cpp:43 */
#define GBL_STEP 0.018f                   /* amd_bcx_body.cpp:47 */
#define GBL_EXT 0.1f                      /* amd_bcx_body.cpp:48 */
#define LCL_STEP 0.6f                     /* amd_bcx_body.cpp:49 */

static float fminr(float a, float b) { return a < b ? a : b; }  /* Math_MinF */
static float fmaxr(float a, float b) { return a > b ? a : b; }  /* Math_MaxF */

static int chan_bits(int ch) { return ch == CH_G ? 6 : 5; }

/* ---------------------------------------------------------------- ramps --- */

/* MkRmpOnGrid, amd_bcx_body.cpp:122-151 (min 0, max 255). */
static void snap_grid(float out[3][2], float in[3][2])
{
    for (int ch = 0; ch < 3; ++ch) {
        const float f1 = (float)(1 << chan_bits(ch));
        const float f0 = (float)(1 << (8 - chan_bits(ch)));
        for (int e = 0; e < 2; ++e) {
            float v = floorf(in[ch][e]);
            if (v <= 0.f) {
                v = 0.f;
            } else {
                v += floorf(128.f / f1) - floorf(v / f1);
                v = fminr(v, 255.f);
            }
            out[ch][e] = floorf(v / f0) * f0;
        }
    }
}

/* MkWkRmpPts, amd_bcx_body.cpp:157-181: bit replication of grid endpoints. */
static int expand_grid(float out[3][2], float in[3][2])
{
    int flat = 1;
    for (int ch = 0; ch < 3; ++ch)
        flat &= (in[ch][0] == in[ch][1]);
    for (int ch = 0; ch < 3; ++ch) {
        const float f = (float)(1 << chan_bits(ch));
        for (int e = 0; e < 2; ++e) {
            float v = in[ch][e] + floorf(in[ch][e] / f);
            v = fmaxr(v, 0.f);
            out[ch][e] = fminr(v, 255.f);
        }
    }
    return flat;
}

/* BldClrRmp, amd_bcx_body.cpp:188-197 (dwRndAmount :183). */
static void chan_ramp(float r[4], const float ends[2], int n)
{
    const float rnd = (n == 4) ? 1.f : 0.f;
    r[0] = ends[0];
    r[n - 1] = ends[1];
    if (n & 1)
        r[n] = 1000000.f;
    for (int e = 1; e < n - 1; ++e)
        r[e] = floorf((r[0] * (float)(n - 1 - e) + r[n - 1] * (float)e + rnd) / (float)(n - 1));
}

static void colour_ramp(float r[3][4], float ends[3][2], int n)
{
    for (int ch = 0; ch < 3; ++ch)
        chan_ramp(r[ch], ends[ch], n);
}

/* ClstrErr with weights, amd_bcx_body.cpp:214-255. */
static float ramp_fit_error(float blk[16][4], const float rpt[16], float r[3][4],
                            int ncol, int n, int flat, const float w[3])
{
    float err = 0.f;
    const int nr = flat ? 1 : n;
    for (int i = 0; i < ncol; ++i) {
        float best = 99999999999.f;
        for (int k = 0; k < nr; ++k) {
            float d = (blk[i][CH_R] - r[CH_R][k]) * (blk[i][CH_R] - r[CH_R][k]) * w[0] +
                      (blk[i][CH_G] - r[CH_G][k]) * (blk[i][CH_G] - r[CH_G][k]) * w[1] +
                      (blk[i][CH_B] - r[CH_B][k]) * (blk[i][CH_B] - r[CH_B][k]) * w[2];
            if (d < best)
                best = d;
        }
        err += best * rpt[i];
    }
    return err;
}

/* ClstrIntnl with weights, amd_bcx_body.cpp:258-317. */
static float assign_indices(float blk[16][4], uint8_t idx[16], float r[3][4], int n,
                            int flat, const float w[3], int use_alpha)
{
    float err = 0.f;
    const int nr = flat ? 1 : n;
    for (int i = 0; i < 16; ++i) {
        uint32_t abits;
        memcpy(&abits, &blk[i][CH_A], 4);
        if (use_alpha && abits == 0) {
            idx[i] = (uint8_t)n;
            continue;
        }
        float best = 99999999999.f;
        int bi = 0;
        for (int k = 0; k < nr; ++k) {
            float d = (blk[i][CH_R] - r[CH_R][k]) * (blk[i][CH_R] - r[CH_R][k]) * w[0] +
                      (blk[i][CH_G] - r[CH_G][k]) * (blk[i][CH_G] - r[CH_G][k]) * w[1] +
                      (blk[i][CH_B] - r[CH_B][k]) * (blk[i][CH_B] - r[CH_B][k]) * w[2];
            if (d < best) {
                best = d;
                bi = k;
            }
        }
        err += best;
        /* DXT index order: last ramp point -> 1, inner points shift up */
        if (bi == n - 1)
            bi = 1;
        else if (bi)
            bi++;
        idx[i] = (uint8_t)bi;
    }
    return err;
}

/* Clstr -> ClstrBas, amd_bcx_body.cpp:322-378.  blk255 is B,G,R,A x255. */
static float final_cluster(const float blk255[64], uint8_t ep[3][2], uint8_t idx[16], int n,
                           const float w[3], int use_alpha, float thr01)
{
    unsigned c0 = ((unsigned)(ep[CH_R][0] & 0xf8) << 8) | ((unsigned)(ep[CH_G][0] & 0xfc) << 3) |
                  ((unsigned)(ep[CH_B][0] & 0xf8) >> 3);
    unsigned c1 = ((unsigned)(ep[CH_R][1] & 0xf8) << 8) | ((unsigned)(ep[CH_G][1] & 0xfc) << 3) |
                  ((unsigned)(ep[CH_B][1] & 0xf8) >> 3);
    int e0 = 0, e1 = 1;
    if ((!(n & 1) && c0 <= c1) || ((n & 1) && c0 > c1)) {
        e0 = 1;
        e1 = 0;
    }
    float ends[3][2];
    for (int ch = 0; ch < 3; ++ch) {
        ends[ch][0] = (float)ep[ch][e0];
        ends[ch][1] = (float)ep[ch][e1];
    }
    const float thr = thr01 * 255.f;
    float blk[16][4];
    for (int i = 0; i < 16; ++i) {
        blk[i][CH_R] = blk255[i * 4 + 2];
        blk[i][CH_G] = blk255[i * 4 + 1];
        blk[i][CH_B] = blk255[i * 4 + 0];
        blk[i][CH_A] = 0.f;
        if (use_alpha)
            blk[i][CH_A] = (blk255[i * 4 + 3] >= thr) ? 1.f : 0.f;
    }
    float wk[3][2], r[3][4];
    int flat = expand_grid(wk, ends);
    colour_ramp(r, wk, n);
    return assign_indices(blk, idx, r, n, flat, w, use_alpha);
}

/* --------------------------------------------------------- 1-D search --- */

/* RampSrchW, amd_bcx_body.cpp:398-435 (early-out kept verbatim). */
static float proj_ramp_error(const float *prj, const float *perr, const float *rpt,
                             float maxerr, float lo, float hi, int ncol, int n)
{
    float error = 0;
    const float step = (hi - lo) / (float)(n - 1);
    const float step_h = step * (float)0.5;
    const float rstep = (float)1.0f / step;
#ifdef ORC_STATS
    if (orc_bcx_ramp_hook) {
        float run[16] = {0}, acc = 0;
        for (int i = 0; i < ncol; ++i) {
            float v, del;
            if ((del = prj[i] - lo) <= 0)
                v = lo;
            else if (prj[i] - hi >= 0)
                v = hi;
            else
                v = floorf((del + step_h) * rstep) * step + lo;
            float d = prj[i] - v;
            d *= d;
            acc += rpt[i] * d + perr[i];
            run[i] = acc;
        }
        for (int i = ncol; i < 16; ++i) run[i] = acc;
        orc_bcx_ramp_hook(run, perr, maxerr, ncol, n);
    }
#endif
    for (int i = 0; i < ncol; ++i) {
        float v, del;
        if ((del = prj[i] - lo) <= 0)
            v = lo;
        else if (prj[i] - hi >= 0)
            v = hi;
        else
            v = floorf((del + step_h) * rstep) * step + lo;
        float d = prj[i] - v;
        d *= d;
        float e = rpt[i] * d + perr[i];
        error += e;
        if (maxerr < error) {
            error = maxerr;
            break;
        }
    }
    return error;
}

/* FindAxis, amd_bcx_body.cpp:442-570 (nDimensions = 3). */
static void principal_axis(float shifted[16][4], float dir[3], float centre[3], int *small,
                           float blk[16][4], const float rpt[16], int ncol)
{
    float crr[3] = {0, 0, 0}, var[3] = {0, 0, 0};
    dir[0] = dir[1] = dir[2] = 0.f;
    centre[0] = centre[1] = centre[2] = 0.f;
    float npts = 0.f;
    for (int i = 0; i < ncol; ++i) {
        centre[0] += blk[i][0] * rpt[i];
        centre[1] += blk[i][1] * rpt[i];
        centre[2] += blk[i][2] * rpt[i];
        npts += rpt[i];
    }
    centre[0] /= npts;
    centre[1] /= npts;
    centre[2] /= npts;
    for (int i = 0; i < ncol; ++i) {
        shifted[i][0] = blk[i][0] - centre[0];
        shifted[i][1] = blk[i][1] - centre[1];
        shifted[i][2] = blk[i][2] - centre[2];
        for (int j = 0; j < 3; ++j) {
            var[j] += shifted[i][j] * shifted[i][j] * rpt[i];
            crr[j] += shifted[i][j] * shifted[i][(j + 1) % 3] * rpt[i];
        }
    }
    int i0 = 0, i1 = 1, k = 0;
    float mx = 0.f;
    /* EPS / EPS2 macros expand unparenthesised: npts * (2/255) * (2/255) */
    const float eps = npts * (2.f / 255.f) * (2.f / 255.f);
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
    *small = 1;
    for (int j = 0; j < 3; ++j)
        *small &= (var[j] < eps2);
    if (*small)
        return;
    if (k == 1) {
        dir[i0] = 1.f;
    } else if (k == 2) {
        i1 = (var[(i0 + 1) % 3] > 0.f) ? (i0 + 1) % 3 : (i0 + 2) % 3;
        float cr = (i1 == (i0 + 1) % 3) ? crr[i0] : crr[(i0 + 2) % 3];
        dir[i1] = cr / var[i0];
        dir[i0] = 1.f;
    } else {
        float best_det = 100000.f;
        for (int j = 0; j < 3; ++j) {
            float det = var[j] * var[(j + 1) % 3] - crr[j] * crr[j];
            if (best_det < det) {
                best_det = det;
                i0 = j;
            }
        }
        /* 2x2 inverse solve, amd_bcx_body.cpp:541-561 */
        float a = var[(i0 + 1) % 3], b = -crr[i0], c = var[i0];
        float u0 = crr[(i0 + 2) % 3], u1 = crr[(i0 + 1) % 3];
        float s0 = a * u0 + b * u1;
        float s1 = b * u0 + c * u1;
        s0 /= best_det;
        s1 /= best_det;
        dir[i0] = 1.f;
        dir[(i0 + 1) % 3] = 1.f;
        dir[(i0 + 2) % 3] = s0 + s1;
    }
    float len = dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2];
    len = sqrtf(len);
    for (int j = 0; j < 3; ++j)
        dir[j] = (len > 0.f) ? dir[j] / len : 0.f;
}

/* Refine (RefinementSteps per-channel 565 jitter), amd_bcx_body.cpp:582-806.
 * The three channel passes share one body; only the association of the
 * error terms differs per pass and is kept literal. */
static void refine_channels(float out[3][2], float in[3][2], float blk[16][4],
                            const float rpt[16], int ncol, int n, const float w[3], int steps)
{
    const float wr = w[0], wg = w[1], wb = w[2];
    float base[3][2], cur[3][2], wk[3][2], r[3][4];
    for (int e = 0; e < 2; ++e)
        for (int ch = 0; ch < 3; ++ch)
            base[ch][e] = cur[ch][e] = out[ch][e] = in[ch][e];
    int flat = expand_grid(wk, cur);
    colour_ramp(r, wk, n);
    float best = ramp_fit_error(blk, rpt, r, ncol, n, flat, w);
    if (best == 0.f || !steps)
        return;

    float side[4][16];
    const int lo = -(int)fminr((float)steps, 8.f), hi = (int)fminr((float)steps, 8.f);
    /* pass order R, G, B; "other two" error pre-computed per pass */
    static const int pass_ch[3] = {CH_R, CH_G, CH_B};
    for (int pass = 0; pass < 3; ++pass) {
        const int ch = pass_ch[pass];
        if (pass > 0) {
            flat = expand_grid(wk, cur);
            colour_ramp(r, wk, n);
        }
        for (int i = 0; i < ncol; ++i)
            for (int k = 0; k < n; ++k) {
                if (ch == CH_R) {
                    float dg = r[CH_G][k] - blk[i][CH_G], db = r[CH_B][k] - blk[i][CH_B];
                    side[k][i] = dg * dg * wg + db * db * wb;
                } else if (ch == CH_G) {
                    float dr = r[CH_R][k] - blk[i][CH_R], db = r[CH_B][k] - blk[i][CH_B];
                    side[k][i] = dr * dr * wr + db * db * wb;
                } else {
                    float dr = r[CH_R][k] - blk[i][CH_R], dg = r[CH_G][k] - blk[i][CH_G];
                    side[k][i] = dr * dr * wr + dg * dg * wg;
                }
            }
        const float grid = (float)(1 << (8 - chan_bits(ch)));
        const float wc = (ch == CH_R) ? wr : (ch == CH_G) ? wg : wb;
        float b0 = base[ch][0], b1 = base[ch][1];
        for (int a = lo; a <= hi; ++a)
            for (int b = lo; b <= hi; ++b) {
                cur[ch][0] = fminr(fmaxr(base[ch][0] + (float)a * grid, 0.f), 255.f);
                cur[ch][1] = fminr(fmaxr(base[ch][1] + (float)b * grid, 0.f), 255.f);
                flat = expand_grid(wk, cur);
                chan_ramp(r[ch], wk[ch], n);
                float mse = 0.f;
                const int nr = flat ? 1 : n;
                for (int i = 0; i < ncol; ++i) {
                    float m = 10000000.f;
                    for (int k = 0; k < nr; ++k) {
                        float d = r[ch][k] - blk[i][ch];
                        float e = side[k][i] + d * d * wc;
                        m = fminr(m, e);
                    }
                    mse += m * rpt[i];
                }
                if (mse < best) {
                    b0 = cur[ch][0];
                    b1 = cur[ch][1];
                    best = mse;
                }
            }
        cur[ch][0] = b0;
        cur[ch][1] = b1;
    }
    for (int ch = 0; ch < 3; ++ch)
        for (int e = 0; e < 2; ++e)
            out[ch][e] = cur[ch][e];
}

/* Refine3D, amd_bcx_body.cpp:808-932 (b3DRefinement): joint jitter of the six
 * endpoint coordinates, G outermost, then B, then R. */
static void refine_3d(float out[3][2], float in0[3][2], float blk[16][4], const float rpt[16], int ncol, int n,
                      const float w[3], int steps)
{
    const float wr = w[0], wg = w[1], wb = w[2];
    float rmp[3][4], inp0[3][2], inp[3][2], wk[3][2];
    for (int k = 0; k < 2; ++k)
        for (int j = 0; j < 3; ++j)
            inp0[j][k] = inp[j][k] = out[j][k] = in0[j][k];
    int eq = expand_grid(wk, inp);
    colour_ramp(rmp, wk, n);
    float best = ramp_fit_error(blk, rpt, rmp, ncol, n, eq, w);
    if (best == 0.f || !steps)
        return;
    const int lo = 0 - (int)fminr((float)steps, 8.f), hi = (int)fminr((float)steps, 8.f);
    const float fr = (float)(1 << (8 - chan_bits(CH_R))), fg = (float)(1 << (8 - chan_bits(CH_G))),
                fb = (float)(1 << (8 - chan_bits(CH_B)));
    for (int g0 = lo; g0 <= hi; g0++) {
        inp[CH_G][0] = fminr(fmaxr(inp0[CH_G][0] + g0 * fg, 0.f), 255.f);
        for (int g1 = lo; g1 <= hi; g1++) {
            inp[CH_G][1] = fminr(fmaxr(inp0[CH_G][1] + g1 * fg, 0.f), 255.f);
            eq = expand_grid(wk, inp);
            chan_ramp(rmp[CH_G], wk[CH_G], n);
            float errg[4][16];
            for (int i = 0; i < ncol; i++)
                for (int r = 0; r < n; r++) {
                    float dg = rmp[CH_G][r] - blk[i][CH_G];
                    errg[r][i] = dg * dg * wg;
                }
            for (int b0 = lo; b0 <= hi; b0++) {
                inp[CH_B][0] = fminr(fmaxr(inp0[CH_B][0] + b0 * fb, 0.f), 255.f);
                for (int b1 = lo; b1 <= hi; b1++) {
                    inp[CH_B][1] = fminr(fmaxr(inp0[CH_B][1] + b1 * fb, 0.f), 255.f);
                    eq = expand_grid(wk, inp);
                    chan_ramp(rmp[CH_B], wk[CH_B], n);
                    float err[4][16];
                    for (int i = 0; i < ncol; i++)
                        for (int r = 0; r < n; r++) {
                            float db = rmp[CH_B][r] - blk[i][CH_B];
                            err[r][i] = errg[r][i] + db * db * wb;
                        }
                    for (int r0 = lo; r0 <= hi; r0++) {
                        inp[CH_R][0] = fminr(fmaxr(inp0[CH_R][0] + r0 * fr, 0.f), 255.f);
                        for (int r1 = lo; r1 <= hi; r1++) {
                            inp[CH_R][1] = fminr(fmaxr(inp0[CH_R][1] + r1 * fr, 0.f), 255.f);
                            eq = expand_grid(wk, inp);
                            chan_ramp(rmp[CH_R], wk[CH_R], n);
                            float mse = 0.f;
                            const int rl = eq ? 1 : n;
                            for (int k = 0; k < ncol; k++) {
                                float m = 10000000.f;
                                for (int r = 0; r < rl; r++) {
                                    float d = rmp[CH_R][r] - blk[k][CH_R];
                                    float e2 = err[r][k] + d * d * wr;
                                    m = fminr(m, e2);
                                }
                                mse += m * rpt[k];
                            }
                            if (mse < best) {
                                best = mse;
                                for (int k = 0; k < 2; k++)
                                    for (int j = 0; j < 3; j++)
                                        out[j][k] = inp[j][k];
                            }
                        }
                    }
                }
            }
        }
    }
}

/* CompressRGBBlockX, amd_bcx_body.cpp:937-1203.  blkin: unique colours x255. */
static void fit_endpoints(float result[3][2], float blkin[16][4], const float rpt[16],
                          int nuniq, int n, int steps, const float w[3], int b3d)
{
    float blk[16][4], sh[16][4], dir0[3], mid[3];
    float rc[3][2];
    for (int i = 0; i < nuniq; ++i)
        for (int j = 0; j < 3; ++j)
            blk[i][j] = blkin[i][j] / 255.f;
    int done = 0;
    if (nuniq <= 2) {
        for (int j = 0; j < 3; ++j) {
            rc[j][0] = blkin[0][j];
            rc[j][1] = blkin[nuniq - 1][j];
        }
        done = 1;
    }
    if (!done) {
        int small = 1;
        principal_axis(sh, dir0, mid, &small, blk, rpt, nuniq);
        if (small) {
            for (int j = 0; j < 3; ++j) {
                rc[j][0] = blkin[0][j];
                rc[j][1] = blkin[nuniq - 1][j];
            }
            done = 1;
        }
    }
    if (!done) {
        float err_g = 10000000.f;
        float dir[3] = {dir0[0], dir0[1], dir0[2]}, dir_g[3] = {0, 0, 0}, pos_g[2] = {0, 0};
        float prj0[16], prj[16], perr[16], prem[16], ridx[16];
        for (;;) {
#ifdef ORC_STATS
            orc_bcx_stat[n == 3 ? 0 : 1]++;   /* axis-loop iterations of the 3- / 4-colour search */
#endif
            float bnd[2] = {1000.f, -1000.f};
            for (int i = 0; i < 16; ++i)
                prj0[i] = prj[i] = perr[i] = prem[i] = 0.f;
            for (int i = 0; i < nuniq; ++i) {
                prj0[i] = prj[i] = sh[i][0] * dir[0] + sh[i][1] * dir[1] + sh[i][2] * dir[2];
                perr[i] = (sh[i][0] - dir[0] * prj[i]) * (sh[i][0] - dir[0] * prj[i]) +
                          (sh[i][1] - dir[1] * prj[i]) * (sh[i][1] - dir[1] * prj[i]) +
                          (sh[i][2] - dir[2] * prj[i]) * (sh[i][2] - dir[2] * prj[i]);
                bnd[0] = fminr(bnd[0], prj[i]);
                bnd[1] = fmaxr(bnd[1], prj[i]);
            }
            float scl[2];
            scl[0] = bnd[0] - (bnd[1] - bnd[0]) * 0.125f;
            scl[1] = bnd[1] + (bnd[1] - bnd[0]) * 0.125f;
            const float scl2 = (scl[1] - scl[0]) * (scl[1] - scl[0]);
            const float over = 1.f / (scl[1] - scl[0]);
            for (int i = 0; i < nuniq; ++i) {
                prj[i] = (prj[i] - scl[0]) * over;
                prem[i] = rpt[i] * scl2;
            }
            for (int k = 0; k < 2; ++k)
                bnd[k] = (bnd[k] - scl[0]) * over;
            float err = BCX_MAX_ERROR;
            const float stp = 0.025f;
            const float ls = (bnd[0] - 2.f * stp > 0.f) ? bnd[0] - 2.f * stp : 0.f;
            const float he = (bnd[1] + 2.f * stp < 1.f) ? bnd[1] + 2.f * stp : 1.f;
            float pos[2] = {0, 0};
            float lp = ls;
            for (int l = 0; l < 8; ++l, lp += stp) {
                float hp = he;
                for (int h = 0; h < 8; ++h, hp -= stp) {
                    float e = proj_ramp_error(prj, perr, prem, err, lp, hp, nuniq, n);
                    if (e < err) {
                        err = e;
                        pos[0] = lp;
                        pos[1] = hp;
                    }
                }
            }
            for (int k = 0; k < 2; ++k)
                pos[k] = pos[k] * (scl[1] - scl[0]) + scl[0];
            if ((double)err + 0.001 < (double)err_g) {
                err_g = err;
                dir_g[0] = dir[0];
                dir_g[1] = dir[1];
                dir_g[2] = dir[2];
                pos_g[0] = pos[0];
                pos_g[1] = pos[1];
                const float step = (pos[1] - pos[0]) / (float)(n - 1);
                const float step_h = step * (float)0.5;
                const float rstep = (float)1.0f / step;
                const float over_n = 1.f / (float)(n - 1);
                const float avg = (float)(n - 1) / 2.f;
                for (int i = 0; i < nuniq; ++i) {
                    float del;
                    if ((del = prj0[i] - pos[0]) <= 0)
                        ridx[i] = 0.f;
                    else if (prj0[i] - pos[1] >= 0)
                        ridx[i] = (float)(n - 1);
                    else
                        ridx[i] = floorf((del + step_h) * rstep);
                    ridx[i] = (ridx[i] - avg) * over_n;
                }
                float crs[3] = {0, 0, 0}, len = 0.f;
                for (int i = 0; i < nuniq; ++i) {
                    const float pm = ridx[i] * rpt[i];
                    len += ridx[i] * pm;
                    for (int j = 0; j < 3; ++j)
                        crs[j] += sh[i][j] * pm;
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
            } else {
                break;
            }
        }
        for (int k = 0; k < 2; ++k)
            for (int j = 0; j < 3; ++j)
                rc[j][k] = (pos_g[k] * dir_g[j] + mid[j]) * 255.f;
    }
    float grid[3][2];
    snap_grid(grid, rc);
    if (b3d)
        refine_3d(result, grid, blkin, rpt, nuniq, n, w, steps);
    else
        refine_channels(result, grid, blkin, rpt, nuniq, n, w, steps);
}

static int rgb_key_less(const float *a, const float *b)
{
    /* QSortFloatCmp (amd_bcx_body.cpp:103-117): R, G, B bit patterns */
    uint32_t ka[3], kb[3];
    memcpy(ka, a, 12);
    memcpy(kb, b, 12);
    if (ka[2] != kb[2]) return ka[2] < kb[2];
    if (ka[1] != kb[1]) return ka[1] < kb[1];
    return ka[0] < kb[0];
}

/* CompRGBABlock, amd_bcx_body.cpp:1209-1297.  Returns FLT_MAX (as float) when
 * a 4-colour ramp is requested for a block with transparent texels. */
static float comp_rgba_block(const float *in, uint8_t ep[3][2], uint8_t idx[16], int n,
                             int steps, const float w[3], int use_alpha, float thr01, int b3d)
{
    float rec[16][4];
    int ncol = 0;
    for (int i = 0; i < 16; ++i) {
        if (!use_alpha || in[i * 4 + 3] >= thr01) {
            rec[ncol][0] = in[i * 4 + 2];
            rec[ncol][1] = in[i * 4 + 1];
            rec[ncol][2] = in[i * 4 + 0];
            rec[ncol][3] = 0.f;
            ncol++;
        }
    }
    if (!ncol) {
        for (int ch = 0; ch < 3; ++ch) {
            ep[ch][0] = 0;
            ep[ch][1] = 0xff;
        }
        memset(idx, 0xff, 16);
        return 0.f;
    }
    if (ncol != 16 && use_alpha && !(n & 1))
        return FLT_MAX;
    /* sort (insertion, key-equal records are identical) then dedupe */
    for (int i = 1; i < ncol; ++i) {
        float t[4];
        memcpy(t, rec[i], 16);
        int j = i - 1;
        while (j >= 0 && rgb_key_less(t, rec[j])) {
            memcpy(rec[j + 1], rec[j], 16);
            --j;
        }
        memcpy(rec[j + 1], t, 16);
    }
    float uniq[16][4], rpt[16];
    memset(uniq, 0, sizeof(uniq));
    memset(rpt, 0, sizeof(rpt));
    int nu = 0;
    memcpy(uniq[0], rec[0], 16);
    rpt[0] = 1.f;
    for (int i = 1; i < ncol; ++i) {
        if (memcmp(uniq[nu], rec[i], 16) != 0) {
            nu++;
            memcpy(uniq[nu], rec[i], 16);
            rpt[nu] = 1.f;
        } else {
            rpt[nu] += 1.f;
        }
    }
    nu++;
    for (int i = 0; i < nu; ++i)
        for (int j = 0; j < 4; ++j)
            uniq[i][j] = (float)((double)uniq[i][j] * 255.0);
    float res[3][2];
    fit_endpoints(res, uniq, rpt, nu, n, steps, w, b3d);
    for (int ch = 0; ch < 3; ++ch)
        for (int e = 0; e < 2; ++e)
            ep[ch][e] = (uint8_t)res[ch][e];
    float b255[64];
    for (int i = 0; i < 16; ++i) {
        b255[i * 4 + 0] = in[i * 4 + 2] * 255.0f;
        b255[i * 4 + 1] = in[i * 4 + 1] * 255.0f;
        b255[i * 4 + 2] = in[i * 4 + 0] * 255.0f;
        b255[i * 4 + 3] = in[i * 4 + 3] * 255.0f;
    }
    return final_cluster(b255, ep, idx, n, w, use_alpha, thr01);
}

/* Image_CompressAMDBC1Block, amd_bcx_helpers.cpp:51-105 (non-adaptive
 * weights block_utils.cpp:162-173; b3DRefinement -> Refine3D in the _ex form). */
void orc_bc1_block(const float in[64], int refinement_steps, float alpha_threshold01, uint8_t out8[8])
{
    orc_bc1_block_ex(in, refinement_steps, alpha_threshold01, 0, out8);
}

void orc_bc1_block_ex(const float in[64], int refinement_steps, float alpha_threshold01, int b3d, uint8_t out8[8])
{
    const float w[3] = {0.3086f, 0.6094f, 0.0820f};
    uint8_t ep[2][3][2], idx[2][16];
    const int use_alpha = alpha_threshold01 > 0.0f;
    double e3 = comp_rgba_block(in, ep[0], idx[0], 3, refinement_steps, w, use_alpha, alpha_threshold01, b3d);
    double e4 = (e3 == 0.0) ? FLT_MAX
                            : comp_rgba_block(in, ep[1], idx[1], 4, refinement_steps, w, use_alpha,
                                              alpha_threshold01, b3d);
    const int m = (e3 <= e4) ? 0 : 1;
    unsigned c0 = ((unsigned)(ep[m][CH_R][0] >> 3) << 11) | ((unsigned)(ep[m][CH_G][0] >> 2) << 5) |
                  (unsigned)(ep[m][CH_B][0] >> 3);
    unsigned c1 = ((unsigned)(ep[m][CH_R][1] >> 3) << 11) | ((unsigned)(ep[m][CH_G][1] >> 2) << 5) |
                  (unsigned)(ep[m][CH_B][1] >> 3);
    uint32_t w0, w1 = 0;
    if ((m == 1 && c0 <= c1) || (m == 0 && c0 > c1))
        w0 = c1 | (c0 << 16);
    else
        w0 = c0 | (c1 << 16);
    for (int i = 0; i < 16; ++i)
        w1 |= (uint32_t)((uint64_t)idx[m][i] << (2 * i));
    memcpy(out8, &w0, 4);
    memcpy(out8 + 4, &w1, 4);
}

/* Colour half of BC2/BC3: Image_CompressAMDRGBSingleModeBlock
 * (amd_bcx_helpers.cpp:142-181).  The reference's CompRGBBlock
 * (amd_bcx_body.cpp:1299-1365) is undefined behaviour (stride-4 reads past its
 * 48-float input, endpoints fitted in R,G,B but clustered in B,G,R order), so
 * this restates its intent -- CompRGBABlock's 4-colour fit with alpha ignored
 * -- packed with c0 > c1 as :164-171.  Parity of this half is unpinned (no
 * reference output exists to pin it); the alpha halves are pinned by the BC4
 * restatement they share. */
void orc_rgb4_block(const float in[64], int refinement_steps, int b3d, uint8_t out8[8])
{
    const float w[3] = {0.3086f, 0.6094f, 0.0820f};
    uint8_t ep[3][2], idx[16];
    comp_rgba_block(in, ep, idx, 4, refinement_steps, w, 0, 0.f, b3d);
    unsigned c0 = ((unsigned)(ep[CH_R][0] >> 3) << 11) | ((unsigned)(ep[CH_G][0] >> 2) << 5) |
                  (unsigned)(ep[CH_B][0] >> 3);
    unsigned c1 = ((unsigned)(ep[CH_R][1] >> 3) << 11) | ((unsigned)(ep[CH_G][1] >> 2) << 5) |
                  (unsigned)(ep[CH_B][1] >> 3);
    uint32_t w0 = c0 <= c1 ? (c1 | (c0 << 16)) : (c0 | (c1 << 16)), w1 = 0;
    for (int i = 0; i < 16; ++i)
        w1 |= (uint32_t)((uint64_t)idx[i] << (2 * i));
    memcpy(out8, &w0, 4);
    memcpy(out8 + 4, &w1, 4);
}

/* Image_CompressAMDExplictAlphaSingleModeBlock, amd_bcx_helpers.cpp:107-123
 * (float -> byte clamped to [0,255] first: out-of-range is UB there). */
void orc_explicit_alpha_block(const float in[16], uint8_t out8[8])
{
    uint32_t w[2] = {0, 0};
    for (int i = 0; i < 16; ++i) {
        float f = in[i] * 255.0f;
        f = f < 0.f ? 0.f : (f > 255.f ? 255.f : f);
        unsigned a = (unsigned)(uint8_t)f;
        a = (a + ((a >> 4) < 0x8 ? 7 : 8) - (a >> 4)) >> 4;
        if (a > 0xf) a = 0xf;
        w[i < 8 ? 0 : 1] |= a << ((i % 8) * 4);
    }
    memcpy(out8, w, 8);
}

/* ------------------------------------------------------ scalar (BC4) --- */

/* RmpSrch1, amd_bcx_body.cpp:1510-1548. */
static float scalar_ramp_error(const float *v, const float *rpt, float maxerr, float lo, float hi,
                               int nv, int n)
{
    float error = 0;
    const float step = (hi - lo) / (float)(n - 1);
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
        float d = v[i] - q;
        error += d * d * rpt[i];
        if (maxerr < error) {
            error = maxerr;
            break;
        }
    }
    return error;
}

/* Refine1 hill climb, amd_bcx_body.cpp:1555-1607 (SCH_STPS 3, sMvF :580). */
static float scalar_refine(const float *v, const float *rpt, float maxerr, float *lo, float *hi,
                           float mstep, float lo_bnd, float hi_bnd, int nv, int n)
{
    static const float mv[3] = {0.f, -1.f, 1.f};
    float best = maxerr, a = *lo, b = *hi;
    int bm;
    do {
        float ca0 = a, cb0 = b;
        bm = -1;
        for (int m = 0; m < 9; ++m) {
            float ca = a + mstep * mv[m / 3];
            float cb = b + mstep * mv[m % 3];
            ca = fmaxr(ca, lo_bnd);
            cb = fminr(cb, hi_bnd);
            float e = scalar_ramp_error(v, rpt, best, ca, cb, nv, n);
            if (e < best) {
                best = e;
                bm = m;
                ca0 = ca;
                cb0 = cb;
            }
        }
        if (bm != -1) {
            a = ca0;
            b = cb0;
        }
    } while (bm != -1);
    *lo = a;
    *hi = b;
    return best;
}

/* CompBlock1 with _IntPrc 8, _FracPrc 0, _bFixedRamp true,
 * amd_bcx_body.cpp:1633-1832. */
static void scalar_endpoints(float ramp_out[2], const float *blk, int n, int fixed_pts)
{
    float vals[16];
    memcpy(vals, blk, sizeof(vals));
    /* ascending (QSortFCmp :1609-1618); equal floats are interchangeable */
    for (int i = 1; i < 16; ++i) {
        float t = vals[i];
        int j = i - 1;
        while (j >= 0 && (double)(vals[j] - t) > 0.) {
            vals[j + 1] = vals[j];
            --j;
        }
        vals[j + 1] = t;
    }
    float uv[16], ur[16], ramp[2];
    for (int i = 0; i < 16; ++i)
        uv[i] = ur[i] = 0.f;
    float prev = -2.f;
    int nu = 0, need = 1;
    if (fixed_pts) {
        for (int i = 0; i < 16; ++i) {
            if (prev != vals[i]) {
                prev = vals[i];
                if ((double)prev <= 1.5 / 255.) {
                } else if ((double)prev >= 253.5 / 255.) {
                } else {
                    uv[nu] = vals[i];
                    ur[nu] = 1.f;
                    nu++;
                }
            } else if (nu > 0 && uv[nu - 1] == prev) {
                ur[nu - 1] += 1.f;
            }
        }
        if (nu <= 2) {
            if (nu == 2) {
                ramp[0] = floorf(uv[0] * 255.f + 0.5f);
                ramp[1] = floorf(uv[1] * 255.f + 0.5f);
            } else if (nu == 1) {
                ramp[0] = floorf(uv[0] * 255.f + 0.5f);
                ramp[1] = ramp[0] + 1.f;
            } else {
                ramp[0] = 128.f;
                ramp[1] = ramp[0] + 1.f;
            }
            need = 0;
        }
    } else {
        for (int i = 0; i < 16; ++i) {
            if (prev != vals[i]) {
                uv[nu] = prev = vals[i];
                ur[nu] = 1.f;
                nu++;
            } else {
                ur[nu - 1] += 1.f;
            }
        }
        if (nu <= 2) {
            ramp[0] = floorf(uv[0] * 255.f + 0.5f);
            if (nu == 1)
                ramp[1] = ramp[0] + 1.f;
            else
                ramp[1] = floorf(uv[1] * 255.f + 0.5f);
            need = 0;
        }
    }
    if (need) {
        float lo = uv[0], hi = uv[nu - 1];
        float lr = lo, hr = hi, gl = 0, gr = 0;
        float cntr = (lr + hr) / 2;
        float gerr = BCX_MAX_ERROR;
        if (!(hi - lo <= 48.f / 256.f)) {
            float llb = (0.f > lr - GBL_EXT) ? 0.f : lr - GBL_EXT;
            float rrb = (1.f < hr + GBL_EXT) ? 1.f : hr + GBL_EXT;
            float lrb = (cntr < lr + GBL_EXT) ? cntr : lr + GBL_EXT;
            float rlb = (cntr > hr - GBL_EXT) ? cntr : hr - GBL_EXT;
            for (float sl = llb; sl < lrb; sl += GBL_STEP)
                for (float sr = rrb; rlb <= sr; sr -= GBL_STEP) {
                    float e = scalar_ramp_error(uv, ur, gerr, sl, sr, nu, n);
                    if (e < gerr) {
                        gerr = e;
                        gl = sl;
                        gr = sr;
                    }
                }
            lr = gl;
            hr = gr;
        }
        scalar_refine(uv, ur, gerr, &lr, &hr, LCL_STEP / 256.f, 0.f, 1.f, nu, n);
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
    ramp_out[0] = ramp[0];
    ramp_out[1] = ramp[1];
}

/* GetRmp1 + BldRmp1 + Clstr1, amd_bcx_body.cpp:1395-1505.  Mutates ramp
 * (endpoint swap), as the reference does. */
static float scalar_cluster(uint8_t idx[16], const float *blk, float ramp[2], int n, int fixed_pts)
{
    float err = 0.f, pts[16];
    for (int i = 0; i < 16; ++i)
        idx[i] = 0;
    if (ramp[0] == ramp[1])
        return err;
    if ((!fixed_pts && ramp[0] <= ramp[1]) || (fixed_pts && ramp[0] > ramp[1])) {
        float t = ramp[0];
        ramp[0] = ramp[1];
        ramp[1] = t;
    }
    for (int e = n; e < 16; ++e)
        pts[e] = 100000.f;
    pts[0] = ramp[0];
    pts[1] = ramp[1];
    for (int e = 1; e < n - 1; ++e)
        pts[e + 1] = (pts[0] * (float)(n - 1 - e) + pts[1] * (float)e) / (float)(n - 1);
    if (fixed_pts) {
        pts[n] = 0.f;
        pts[n + 1] = 255.f;
    }
    for (int i = 0; i < n; ++i)
        pts[i] = floorf(pts[i] + 0.5f) / 1.f;
    const int np = fixed_pts ? n + 2 : n;
    const float over = 1.f / ((float)(1 << 8) - 1.f);
    for (int i = 0; i < np; ++i)
        pts[i] *= over;
    for (int i = 0; i < 16; ++i) {
        float best = 10000000.f;
        const float a = blk[i];
        for (int j = 0; j < np; ++j) {
            float d = a - pts[j];
            d *= d;
            if (d < best) {
                best = d;
                idx[i] = (uint8_t)j;
            }
        }
        err += best;
    }
    return err;
}

static float scalar_block(const float *blk, uint8_t ep[2], uint8_t idx[16], int n, int fixed_pts)
{
    float ramp[2];
    scalar_endpoints(ramp, blk, n, fixed_pts);
    float err = scalar_cluster(idx, blk, ramp, n, fixed_pts);
    ep[0] = (uint8_t)ramp[0];
    ep[1] = (uint8_t)ramp[1];
    return err;
}

/* EncodeAlphaBlock, amd_bcx_helpers.cpp:32-46 (48 index bits, LSB first). */
static void pack_bc4(uint8_t out[8], const uint8_t ep[2], const uint8_t idx[16])
{
    uint64_t v = (uint64_t)ep[0] | ((uint64_t)ep[1] << 8);
    for (int i = 0; i < 16; ++i)
        v |= (uint64_t)(idx[i] & 7) << (16 + 3 * i);
    memcpy(out, &v, 8);
}

void orc_bc4_block(const float in[16], uint8_t out[8])
{
    uint8_t ep[2][2], idx[2][16];
    float e8 = scalar_block(in, ep[0], idx[0], 8, 0);
    float e6 = (e8 == 0.f) ? FLT_MAX : scalar_block(in, ep[1], idx[1], 6, 1);
    if (e8 <= e6)
        pack_bc4(out, ep[0], idx[0]);
    else
        pack_bc4(out, ep[1], idx[1]);
}

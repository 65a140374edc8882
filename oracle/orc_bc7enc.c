/*
 * orc_bc7enc.c -- CPU restatement of the bc7enc16 BC7 encoder, the reference's
 * "fast" BC7 path (src/richgel999_bc7enc16.cpp, reached from
 * ImageCompress_Compress(Image_CT_DXBC7, fast=true), imagecompress.cpp:34-36).
 *
 * TEST INFRASTRUCTURE ONLY (see bcn_oracle.h): the parity checker of the HIP
 * kernel in gfx_imagecompress_amd/csrc/gic_bc7enc.hip.  Subsets are kept as
 * compacted texel lists here, as the reference keeps them, so that this
 * restatement and the GPU's masked-texel formulation are independent.
 *
 * Every float expression keeps the reference's types and association order
 * (built with -ffp-contract=off).  Tables: bc7enc_tables.h (generated from the
 * reference's literals by tools/gen_bc7enc_tables.py) and the BPTC shapes of
 * bc7_tables.h.
 *
 * One deliberate choice: handle_alpha_block (:1390-1420) never sets
 * m_endpoints_share_pbit, which bc7enc16_compress_block (:1523) leaves
 * uninitialised on the stack -- undefined behaviour.  Mode 6 has one p-bit per
 * endpoint, and the opaque path sets the flag to false (:1434), so false is
 * used for alpha blocks too; parity of alpha blocks against the reference is
 * unpinned by construction.
 */
#include "bcn_oracle.h"

#include <math.h>
#include <stdint.h>
#include <string.h>

#include "bc7_tables.h"
#include "bc7enc_tables.h"

typedef struct { uint8_t c[4]; } px4;   /* color_quad_u8 */
typedef struct { float v[4]; } v4;      /* vec4F */

static const uint32_t kW3[8] = {0, 9, 18, 27, 37, 46, 55, 64};                               /* :130 */
static const uint32_t kW4[16] = {0, 4, 9, 13, 17, 21, 26, 30, 34, 38, 43, 47, 51, 55, 60, 64};  /* :131 */

static float bits_f(uint32_t u)
{
    float f;
    memcpy(&f, &u, 4);
    return f;
}

static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
static float clampf(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }
static float sat(float v) { return clampf(v, 0, 1.0f); }
static float maxf_r(float a, float b) { return a > b ? a : b; }

static v4 v4_of(const px4 *p)
{
    v4 r = {{p->c[0], p->c[1], p->c[2], p->c[3]}};
    return r;
}
static float v4_dot(const v4 *a, const v4 *b)
{
    return a->v[0] * b->v[0] + a->v[1] * b->v[1] + a->v[2] * b->v[2] + a->v[3] * b->v[3];
}
static void v4_norm(v4 *a)   /* vec4F_normalize_in_place :127 */
{
    float s = a->v[0] * a->v[0] + a->v[1] * a->v[1] + a->v[2] * a->v[2] + a->v[3] * a->v[3];
    if (s != 0.0f) {
        s = 1.0f / sqrtf(s);
        for (int k = 0; k < 4; ++k) a->v[k] *= s;
    }
}
static v4 v4_scale(const v4 *a, float s)
{
    v4 r = {{a->v[0] * s, a->v[1] * s, a->v[2] * s, a->v[3] * s}};
    return r;
}

/* ---- settings (bc7enc16_compress_block_params, richgel999_bc7enc16.h:17-63;
 *      Image_CompressRichGel999BC7enc16, richgel999_bc7enc16.cpp:73-97) ---- */
typedef struct {
    uint32_t max_parts, uber;
    int perceptual, lsq, filterbank;
    uint32_t w[4];   /* error weights after bc7enc16_compress_block's scaling (:1524-1535) */
} cfg_t;

static void make_cfg(int fast, int perceptual, cfg_t *c)
{
    uint32_t base[4];
    c->max_parts = 64;
    c->lsq = 1;
    c->filterbank = 1;
    c->uber = fast ? 0 : 4;
    c->perceptual = perceptual;
    if (perceptual) {
        base[0] = 128, base[1] = 64, base[2] = 16, base[3] = 32;
        const float pr = (.5f / (1.0f - .2126f)) * (.5f / (1.0f - .2126f));
        const float pb = (.5f / (1.0f - .0722f)) * (.5f / (1.0f - .0722f));
        c->w[0] = (uint32_t)(int)(base[0] * 4.0f);
        c->w[1] = (uint32_t)(int)(base[1] * 4.0f * pr);
        c->w[2] = (uint32_t)(int)(base[2] * 4.0f * pb);
        c->w[3] = base[3] * 4;
    } else {
        c->w[0] = c->w[1] = c->w[2] = c->w[3] = 1;
    }
}

/* g_bc7_mode_1_optimal_endpoints (:162-195): for each 8-bit value and p-bit,
 * the 6-bit endpoint pair whose selector-2 interpolant is closest. */
typedef struct { uint16_t err; uint8_t lo, hi; } one_col;
static one_col g_one[256][2];
static int g_one_ready;

static void init_one_colour(void)
{
    if (g_one_ready) return;
    for (int v = 0; v < 256; ++v)
        for (int p = 0; p < 2; ++p) {
            one_col best = {0xffff, 0, 0};
            for (int l = 0; l < 64; ++l) {
                uint32_t lo = (uint32_t)((l << 1) | p) << 1;
                lo |= lo >> 7;
                for (int h = 0; h < 64; ++h) {
                    uint32_t hi = (uint32_t)((h << 1) | p) << 1;
                    hi |= hi >> 7;
                    const int k = (int)((lo * (64 - kW3[2]) + hi * kW3[2] + 32) >> 6);
                    const int e = (k - v) * (k - v);
                    if (e < best.err) {
                        best.err = (uint16_t)e;
                        best.lo = (uint8_t)l;
                        best.hi = (uint8_t)h;
                    }
                }
            }
            g_one[v][p] = best;
        }
    g_one_ready = 1;
}

/* ---- one subset problem (color_cell_compressor_params / _results :282-305) ---- */
typedef struct {
    uint32_t n;
    const px4 *px;
    uint32_t nsel;
    const uint32_t *selw;   /* integer weights /64 */
    const float *selx;      /* 4 floats per selector */
    uint32_t cbits;
    int alpha, share_pbit, perceptual;
    const uint32_t *w;
} cell_in;

typedef struct {
    uint64_t err;
    px4 lo, hi;
    uint32_t pb[2];
    uint8_t sel[16];
} cell_out;

static px4 expand(const px4 *q, const cell_in *ci)   /* scale_color :307-323 (modes 1/6 have p-bits) */
{
    const uint32_t n = ci->cbits + 1;
    px4 r;
    for (int k = 0; k < 4; ++k) {
        uint32_t v = (uint32_t)q->c[k] << (8 - n);
        r.c[k] = (uint8_t)(v | (v >> n));
    }
    return r;
}

/* compute_color_distance_rgb/_rgba :325-355 */
static uint64_t dist(const px4 *a, const px4 *b, int perceptual, int with_alpha, const uint32_t *w)
{
    int d0, d1, d2;
    if (perceptual) {
        const int l1 = a->c[0] * 109 + a->c[1] * 366 + a->c[2] * 37;
        const int l2 = b->c[0] * 109 + b->c[1] * 366 + b->c[2] * 37;
        d0 = (l1 - l2) >> 8;
        d1 = ((((int)a->c[0] << 9) - l1) - (((int)b->c[0] << 9) - l2)) >> 8;
        d2 = ((((int)a->c[2] << 9) - l1) - (((int)b->c[2] << 9) - l2)) >> 8;
    } else {
        d0 = (int)a->c[0] - (int)b->c[0];
        d1 = (int)a->c[1] - (int)b->c[1];
        d2 = (int)a->c[2] - (int)b->c[2];
    }
    uint64_t e = w[0] * (uint32_t)(d0 * d0) + w[1] * (uint32_t)(d1 * d1) + w[2] * (uint32_t)(d2 * d2);
    if (with_alpha) {
        const int da = (int)a->c[3] - (int)b->c[3];
        e += w[3] * (uint32_t)(da * da);
    }
    return e;
}

/* pack_mode1_to_one_color :357-403 */
static uint64_t one_colour(const cell_in *ci, cell_out *co, uint32_t r, uint32_t g, uint32_t b, uint8_t *sel)
{
    uint32_t best = 0xffffffffu, bp = 0;
    for (uint32_t p = 0; p < 2; ++p) {
        const uint32_t e = (uint32_t)g_one[r][p].err + g_one[g][p].err + g_one[b][p].err;
        if (e < best) best = e, bp = p;
    }
    const one_col *er = &g_one[r][bp], *eg = &g_one[g][bp], *eb = &g_one[b][bp];
    co->lo.c[0] = er->lo, co->lo.c[1] = eg->lo, co->lo.c[2] = eb->lo, co->lo.c[3] = 0;
    co->hi.c[0] = er->hi, co->hi.c[1] = eg->hi, co->hi.c[2] = eb->hi, co->hi.c[3] = 0;
    co->pb[0] = bp;
    co->pb[1] = 0;
    memset(sel, 2, ci->n);
    px4 q;
    for (int k = 0; k < 3; ++k) {
        uint32_t lo = ((uint32_t)(co->lo.c[k] << 1) | bp) << 1;
        lo |= lo >> 7;
        uint32_t hi = ((uint32_t)(co->hi.c[k] << 1) | bp) << 1;
        hi |= hi >> 7;
        q.c[k] = (uint8_t)((lo * (64 - kW3[2]) + hi * kW3[2] + 32) >> 6);
    }
    q.c[3] = 255;
    uint64_t tot = 0;
    for (uint32_t i = 0; i < ci->n; ++i) tot += dist(&q, &ci->px[i], ci->perceptual, 0, ci->w);
    co->err = tot;
    return tot;
}

/* evaluate_solution :405-572 */
static void evaluate(const px4 *lo, const px4 *hi, const uint32_t pb[2], const cell_in *ci, cell_out *co)
{
    const uint32_t p0 = pb[0], p1 = ci->share_pbit ? pb[0] : pb[1];
    px4 qlo, qhi;
    for (int k = 0; k < 4; ++k) {
        qlo.c[k] = (uint8_t)((lo->c[k] << 1) | p0);
        qhi.c[k] = (uint8_t)((hi->c[k] << 1) | p1);
    }
    const px4 a = expand(&qlo, ci), b = expand(&qhi, ci);
    const uint32_t N = ci->nsel;
    const int nc = ci->alpha ? 4 : 3;
    px4 ramp[16];
    memset(ramp, 0, sizeof(ramp));
    ramp[0] = a;
    ramp[N - 1] = b;
    for (uint32_t s = 1; s + 1 < N; ++s)
        for (int k = 0; k < nc; ++k)
            ramp[s].c[k] = (uint8_t)((a.c[k] * (64 - ci->selw[s]) + b.c[k] * ci->selw[s] + 32) >> 6);

    uint8_t tmp[16];
    uint64_t tot = 0;
    if (!ci->perceptual) {
        const int dr = b.c[0] - a.c[0], dg = b.c[1] - a.c[1], db = b.c[2] - a.c[2];
        const int da = ci->alpha ? b.c[3] - a.c[3] : 0;
        const float f = ci->alpha ? N / (float)(dr * dr + dg * dg + db * db + da * da + .00000125f)
                                  : N / (float)(dr * dr + dg * dg + db * db + .00000125f);
        for (uint32_t i = 0; i < ci->n; ++i) {
            const px4 *c = &ci->px[i];
            int dot = (c->c[0] - a.c[0]) * dr + (c->c[1] - a.c[1]) * dg + (c->c[2] - a.c[2]) * db;
            if (ci->alpha) dot += (c->c[3] - a.c[3]) * da;
            int s = (int)((float)dot * f + .5f);
            s = clampi(s, 1, (int)N - 1);
            const uint64_t e0 = dist(&ramp[s - 1], c, 0, ci->alpha, ci->w);
            const uint64_t e1 = dist(&ramp[s], c, 0, ci->alpha, ci->w);
            /* rgba: ties keep s (err1 > err0 moves down, :479); rgb: err0 < err1 moves down (:508) */
            if (e0 < e1) {
                tot += e0;
                --s;
            } else {
                tot += e1;
            }
            tmp[i] = (uint8_t)s;
        }
    } else {
        for (uint32_t i = 0; i < ci->n; ++i) {
            uint64_t be = UINT64_MAX;
            uint32_t bs = 0;
            for (uint32_t s = 0; s < N; ++s) {
                const uint64_t e = dist(&ramp[s], &ci->px[i], 1, ci->alpha, ci->w);
                if (e < be) be = e, bs = s;
            }
            tot += be;
            tmp[i] = (uint8_t)bs;
        }
    }
    if (tot < co->err) {
        co->err = tot;
        co->lo = *lo;
        co->hi = *hi;
        co->pb[0] = pb[0];
        co->pb[1] = pb[1];
        memcpy(co->sel, tmp, ci->n);
    }
}

static int px_ne(const px4 *a, const px4 *b)
{
    return a->c[0] != b->c[0] || a->c[1] != b->c[1] || a->c[2] != b->c[2] || a->c[3] != b->c[3];
}

/* find_optimal_solution :606-729 (both bc7enc16 modes carry p-bits; fixDegenerateEndpoints
 * :574-604 acts on mode 1 only) */
static uint64_t fit(int mode, v4 xl, v4 xh, const cell_in *ci, cell_out *co)
{
    for (int k = 0; k < 4; ++k) xl.v[k] = sat(xl.v[k]), xh.v[k] = sat(xh.v[k]);
    const int iscalep = (1 << (ci->cbits + 1)) - 1;
    const float scalep = (float)iscalep;
    const int ncomp = ci->alpha ? 4 : 3;
    uint32_t bpb[2] = {0, 0};
    px4 bmin = {{0}}, bmax = {{0}};
    if (!ci->share_pbit) {
        float be0 = 1e+9, be1 = 1e+9;
        for (int p = 0; p < 2; ++p) {
            px4 qa, qb;
            for (int k = 0; k < 4; ++k) {
                qa.c[k] = (uint8_t)clampi(((int)((xl.v[k] * scalep - p) / 2.0f + .5f)) * 2 + p, p, iscalep - 1 + p);
                qb.c[k] = (uint8_t)clampi(((int)((xh.v[k] * scalep - p) / 2.0f + .5f)) * 2 + p, p, iscalep - 1 + p);
            }
            const px4 sa = expand(&qa, ci), sb = expand(&qb, ci);
            float e0 = 0, e1 = 0;
            for (int k = 0; k < ncomp; ++k) {
                const float t0 = sa.c[k] - xl.v[k] * 255.0f, t1 = sb.c[k] - xh.v[k] * 255.0f;
                e0 += t0 * t0;
                e1 += t1 * t1;
            }
            if (e0 < be0) {
                be0 = e0, bpb[0] = (uint32_t)p;
                for (int k = 0; k < 4; ++k) bmin.c[k] = qa.c[k] >> 1;
            }
            if (e1 < be1) {
                be1 = e1, bpb[1] = (uint32_t)p;
                for (int k = 0; k < 4; ++k) bmax.c[k] = qb.c[k] >> 1;
            }
        }
    } else {
        float be = 1e+9;
        for (int p = 0; p < 2; ++p) {
            px4 qa, qb;
            for (int k = 0; k < 4; ++k) {
                qa.c[k] = (uint8_t)clampi(((int)((xl.v[k] * scalep - p) / 2.0f + .5f)) * 2 + p, p, iscalep - 1 + p);
                qb.c[k] = (uint8_t)clampi(((int)((xh.v[k] * scalep - p) / 2.0f + .5f)) * 2 + p, p, iscalep - 1 + p);
            }
            const px4 sa = expand(&qa, ci), sb = expand(&qb, ci);
            float e = 0;
            for (int k = 0; k < ncomp; ++k) {
                const float t0 = (sa.c[k] / 255.0f) - xl.v[k], t1 = (sb.c[k] / 255.0f) - xh.v[k];
                e += t0 * t0 + t1 * t1;
            }
            if (e < be) {
                be = e, bpb[0] = bpb[1] = (uint32_t)p;
                for (int k = 0; k < 4; ++k) bmin.c[k] = qa.c[k] >> 1, bmax.c[k] = qb.c[k] >> 1;
            }
        }
    }
    if (mode == 1) {   /* fixDegenerateEndpoints */
        const uint32_t isc = (uint32_t)(iscalep >> 1);
        for (int k = 0; k < 3; ++k) {
            if (bmin.c[k] != bmax.c[k] || !(fabsf(xl.v[k] - xh.v[k]) > 0.0f)) continue;
            if (bmin.c[k] > (isc >> 1)) {
                if (bmin.c[k] > 0)
                    bmin.c[k]--;
                else if (bmax.c[k] < isc)
                    bmax.c[k]++;
            } else {
                if (bmax.c[k] < isc)
                    bmax.c[k]++;
                else if (bmin.c[k] > 0)
                    bmin.c[k]--;
            }
        }
    }
    if (co->err == UINT64_MAX || px_ne(&bmin, &co->lo) || px_ne(&bmax, &co->hi) || bpb[0] != co->pb[0] ||
        bpb[1] != co->pb[1])
        evaluate(&bmin, &bmax, bpb, ci, co);
    return co->err;
}

/* compute_least_squares_endpoints_rgb/_rgba :197-280 */
static void lsq(const cell_in *ci, const uint8_t *sel, v4 *xl, v4 *xh)
{
    float z00 = 0.0f, z10 = 0.0f, z11 = 0.0f;
    float q00[4] = {0, 0, 0, 0}, t[4] = {0, 0, 0, 0};
    const int nc = ci->alpha ? 4 : 3;
    for (uint32_t i = 0; i < ci->n; ++i) {
        const float *wx = ci->selx + 4 * sel[i];
        z00 += wx[0];
        z10 += wx[1];
        z11 += wx[2];
        const float w = wx[3];
        for (int k = 0; k < nc; ++k) {
            q00[k] += w * ci->px[i].c[k];
            t[k] += ci->px[i].c[k];
        }
    }
    const float z01 = z10;
    float det = z00 * z11 - z01 * z10;
    if (det != 0.0f) det = 1.0f / det;
    const float i00 = z11 * det, i01 = -z01 * det, i10 = -z10 * det, i11 = z00 * det;
    for (int k = 0; k < nc; ++k) {
        const float q10 = t[k] - q00[k];
        xl->v[k] = (float)(i00 * q00[k] + i01 * q10);
        xh->v[k] = (float)(i10 * q00[k] + i11 * q10);
    }
    if (nc == 3) xl->v[3] = 255.0f, xh->v[3] = 255.0f;
}

/* the least-squares refit of a selector set, then a fit (the repeated block of :878-1004) */
static uint64_t refit(int mode, const cell_in *ci, cell_out *co, const uint8_t *sel)
{
    v4 xl = {{0, 0, 0, 0}}, xh = {{0, 0, 0, 0}};
    lsq(ci, sel, &xl, &xh);
    xl = v4_scale(&xl, 1.0f / 255.0f);
    xh = v4_scale(&xh, 1.0f / 255.0f);
    return fit(mode, xl, xh, ci, co);
}

/* color_cell_compression :731-1024 */
static uint64_t cell(int mode, const cell_in *ci, cell_out *co, const cfg_t *cfg)
{
    co->err = UINT64_MAX;
    if (mode == 1) {
        int same = 1;
        for (uint32_t i = 1; i < ci->n && same; ++i)
            same = ci->px[i].c[0] == ci->px[0].c[0] && ci->px[i].c[1] == ci->px[0].c[1] &&
                   ci->px[i].c[2] == ci->px[0].c[2];
        if (same) return one_colour(ci, co, ci->px[0].c[0], ci->px[0].c[1], ci->px[0].c[2], co->sel);
    }
    v4 mean = {{0, 0, 0, 0}}, axis;
    for (uint32_t i = 0; i < ci->n; ++i)
        for (int k = 0; k < 4; ++k) mean.v[k] = mean.v[k] + (float)ci->px[i].c[k];
    const v4 mean_s = v4_scale(&mean, 1.0f / (float)ci->n);
    mean = v4_scale(&mean, 1.0f / (float)(ci->n * 255.0f));
    for (int k = 0; k < 4; ++k) mean.v[k] = sat(mean.v[k]);

    if (ci->alpha) {   /* incremental PCA :773-790 */
        memset(&axis, 0, sizeof(axis));
        for (uint32_t i = 0; i < ci->n; ++i) {
            v4 c = v4_of(&ci->px[i]);
            for (int k = 0; k < 4; ++k) c.v[k] = c.v[k] - mean_s.v[k];
            v4 pr[4];
            for (int r = 0; r < 4; ++r) pr[r] = v4_scale(&c, c.v[r]);
            v4 n = i ? axis : c;
            v4_norm(&n);
            for (int r = 0; r < 4; ++r) axis.v[r] += v4_dot(&pr[r], &n);
        }
        v4_norm(&axis);
    } else {   /* covariance + 3 power steps :795-831 */
        float cv[6] = {0, 0, 0, 0, 0, 0};
        for (uint32_t i = 0; i < ci->n; ++i) {
            const float r = ci->px[i].c[0] - mean_s.v[0];
            const float g = ci->px[i].c[1] - mean_s.v[1];
            const float b = ci->px[i].c[2] - mean_s.v[2];
            cv[0] += r * r, cv[1] += r * g, cv[2] += r * b, cv[3] += g * g, cv[4] += g * b, cv[5] += b * b;
        }
        float vr = .9f, vg = 1.0f, vb = .7f;
        for (int it = 0; it < 3; ++it) {
            float r = vr * cv[0] + vg * cv[1] + vb * cv[2];
            float g = vr * cv[1] + vg * cv[3] + vb * cv[4];
            float b = vr * cv[2] + vg * cv[4] + vb * cv[5];
            float m = maxf_r(maxf_r(fabsf(r), fabsf(g)), fabsf(b));   /* maximumf :108 */
            if (m > 1e-10f) {
                m = 1.0f / m;
                r *= m, g *= m, b *= m;
            }
            vr = r, vg = g, vb = b;
        }
        float len = vr * vr + vg * vg + vb * vb;
        if (len < 1e-10f) {
            memset(&axis, 0, sizeof(axis));
        } else {
            len = 1.0f / sqrtf(len);
            axis.v[0] = vr * len, axis.v[1] = vg * len, axis.v[2] = vb * len, axis.v[3] = 0;
        }
    }
    if (v4_dot(&axis, &axis) < .5f) {
        if (ci->perceptual)
            axis.v[0] = .213f, axis.v[1] = .715f, axis.v[2] = .072f, axis.v[3] = ci->alpha ? .715f : 0;
        else
            axis.v[0] = 1.0f, axis.v[1] = 1.0f, axis.v[2] = 1.0f, axis.v[3] = ci->alpha ? 1.0f : 0;
        v4_norm(&axis);
    }
    float lo = 1e+9f, hi = -1e+9f;
    for (uint32_t i = 0; i < ci->n; ++i) {
        v4 q = v4_of(&ci->px[i]);
        for (int k = 0; k < 4; ++k) q.v[k] = q.v[k] - mean_s.v[k];
        const float d = v4_dot(&q, &axis);
        lo = lo < d ? lo : d;   /* minimumf / maximumf :105,108 */
        hi = hi > d ? hi : d;
    }
    lo *= (1.0f / 255.0f);
    hi *= (1.0f / 255.0f);
    v4 cmin, cmax;
    for (int k = 0; k < 4; ++k) {
        cmin.v[k] = sat(mean.v[k] + axis.v[k] * lo);
        cmax.v[k] = sat(mean.v[k] + axis.v[k] * hi);
    }
    const v4 white = {{1.0f, 1.0f, 1.0f, 1.0f}};
    if (v4_dot(&cmin, &white) > v4_dot(&cmax, &white)) {
        const v4 t = cmin;
        cmin = cmax;
        cmax = t;
    }
    if (!fit(mode, cmin, cmax, ci, co)) return 0;
    if (cfg->lsq && !refit(mode, ci, co, co->sel)) return 0;

    if (cfg->uber > 0) {   /* :896-1006 */
        uint8_t base[16], trial[16];
        memcpy(base, co->sel, ci->n);
        const int maxs = (int)ci->nsel - 1;
        uint32_t smin = 16, smax = 0;
        for (uint32_t i = 0; i < ci->n; ++i) {
            smin = base[i] < smin ? base[i] : smin;
            smax = base[i] > smax ? base[i] : smax;
        }
        for (uint32_t i = 0; i < ci->n; ++i)
            trial[i] = (uint8_t)((base[i] == smin && base[i] < ci->nsel - 1) ? base[i] + 1 : base[i]);
        if (!refit(mode, ci, co, trial)) return 0;
        for (uint32_t i = 0; i < ci->n; ++i) trial[i] = (uint8_t)((base[i] == smax && base[i] > 0) ? base[i] - 1 : base[i]);
        if (!refit(mode, ci, co, trial)) return 0;
        for (uint32_t i = 0; i < ci->n; ++i) {
            uint32_t s = base[i];
            if (s == smin && s < ci->nsel - 1)
                s++;
            else if (s == smax && s > 0)
                s--;
            trial[i] = (uint8_t)s;
        }
        if (!refit(mode, ci, co, trial)) return 0;
        const uint32_t thresh = (ci->n * 56) >> 4;
        if (cfg->uber >= 2 && co->err > thresh) {
            const int Q = cfg->uber >= 4 ? (int)cfg->uber - 2 : 1;
            for (int ly = -Q; ly <= 1; ++ly)
                for (int hy = maxs - 1; hy <= maxs + Q; ++hy) {
                    if (ly == 0 && hy == maxs) continue;
                    for (uint32_t i = 0; i < ci->n; ++i)
                        trial[i] = (uint8_t)clampf(
                            floorf((float)maxs * ((float)base[i] - (float)ly) / ((float)hy - (float)ly) + .5f), 0,
                            (float)maxs);
                    if (!refit(mode, ci, co, trial)) return 0;
                }
        }
    }
    if (mode == 1) {   /* the block mean as one colour :1009-1021 */
        const uint32_t r = (uint32_t)(int)(.5f + mean.v[0] * 255.0f), g = (uint32_t)(int)(.5f + mean.v[1] * 255.0f),
                       b = (uint32_t)(int)(.5f + mean.v[2] * 255.0f);
        cell_out avg = *co;
        uint8_t sel[16];
        const uint64_t e = one_colour(ci, &avg, r, g, b, sel);
        if (e < co->err) {
            *co = avg;
            memcpy(co->sel, sel, ci->n);
            co->err = e;
        }
    }
    return co->err;
}

/* color_cell_compression_est :1026-1162: bounding-box endpoints, 8 selectors by
 * dot-product thresholds.  The reference stops summing once the partial sum
 * exceeds the best so far; its caller only compares with '<', so full sums are
 * equivalent. */
static uint64_t estimate(uint32_t n, const px4 *px, int perceptual, const uint32_t *w)
{
    uint32_t lo[3] = {255, 255, 255}, hi[3] = {0, 0, 0};
    for (uint32_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) {
            if (px[i].c[k] < lo[k]) lo[k] = px[i].c[k];
            if (px[i].c[k] > hi[k]) hi[k] = px[i].c[k];
        }
    px4 ramp[8];
    for (int s = 0; s < 8; ++s)
        for (int k = 0; k < 3; ++k)
            ramp[s].c[k] = s == 0 ? (uint8_t)lo[k]
                         : s == 7 ? (uint8_t)hi[k]
                                  : (uint8_t)((lo[k] * (64 - kW3[s]) + hi[k] * kW3[s] + 32) >> 6);
    const int ar = (int)hi[0] - (int)lo[0], ag = (int)hi[1] - (int)lo[1], ab = (int)hi[2] - (int)lo[2];
    int dots[8], th[7];
    for (int s = 0; s < 8; ++s) dots[s] = ramp[s].c[0] * ar + ramp[s].c[1] * ag + ramp[s].c[2] * ab;
    for (int s = 0; s < 7; ++s) th[s] = (dots[s] + dots[s + 1] + 1) >> 1;
    uint64_t tot = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const int d = ar * px[i].c[0] + ag * px[i].c[1] + ab * px[i].c[2];
        int s = 0;
        for (int k = 6; k >= 0; --k)
            if (d >= th[k]) {
                s = k + 1;
                break;
            }
        if (perceptual) {
            const px4 *e = &ramp[s];
            const int l1 = e->c[0] * 109 + e->c[1] * 366 + e->c[2] * 37;
            const int l2 = px[i].c[0] * 109 + px[i].c[1] * 366 + px[i].c[2] * 37;
            const int dl = (l1 - l2) >> 8;
            const int dcr = ((((int)e->c[0] << 9) - l1) - (((int)px[i].c[0] << 9) - l2)) >> 8;
            const int dcb = ((((int)e->c[2] << 9) - l1) - (((int)px[i].c[2] << 9) - l2)) >> 8;
            const int ie = (int)(w[0] * dl * dl + w[1] * dcr * dcr + w[2] * dcb * dcb);
            tot += ie;
        } else {
            const int dr = ramp[s].c[0] - px[i].c[0], dg = ramp[s].c[1] - px[i].c[1], db = ramp[s].c[2] - px[i].c[2];
            tot += w[0] * (dr * dr) + w[1] * (dg * dg) + w[2] * (db * db);
        }
    }
    return tot;
}

static int shape2_of(int part, int t) { return (int)((kBc7Shape2[part] >> (2 * t)) & 3u); }

/* estimate_partition :1207-1281 */
static int pick_partition(const px4 *px, const cfg_t *cfg)
{
    const uint32_t total = cfg->max_parts < 64 ? cfg->max_parts : 64;
    if (total <= 1) return 0;
    uint64_t best = UINT64_MAX;
    int best_part = 0, key = 0;
    for (uint32_t it = 0; it < total && best > 0; ++it) {
        const int part = kEncPartOrder[it];
        if (cfg->filterbank && it >= 14 && it <= 34 && !(kEncPredictors[part] & (1u << (key + 1)))) {
            if (it == 34) break;
            continue;
        }
        px4 sub[2][16];
        uint32_t cnt[2] = {0, 0};
        for (int t = 0; t < 16; ++t) {
            const int s = shape2_of(part, t);
            sub[s][cnt[s]++] = px[t];
        }
        const uint64_t e = estimate(cnt[0], sub[0], cfg->perceptual, cfg->w) +
                           estimate(cnt[1], sub[1], cfg->perceptual, cfg->w);
        if (e < best) best = e, best_part = part;
        if (part == 34 && best_part != 34) break;
        if (it == 13) key = best_part;
    }
    return best_part;
}

/* ---- block packing (encode_bc7_block :1307-1388) ---- */
typedef struct {
    int mode, part;
    uint8_t sel[16];
    px4 lo[2], hi[2];
    uint32_t pb[2][2];
} block_sol;

static void put_bits(uint8_t *out, uint32_t *pos, uint32_t v, uint32_t n)
{
    for (uint32_t i = 0; i < n; ++i, ++*pos)
        if ((v >> i) & 1u) out[*pos >> 3] |= (uint8_t)(1u << (*pos & 7));
}

static void pack_block(block_sol s, uint8_t out[16])
{
    const int nsub = s.mode == 1 ? 2 : 1;
    const uint32_t ib = s.mode == 1 ? 3 : 4;
    int anchor[2] = {0, -1};
    for (int k = 0; k < nsub; ++k) {
        const int a = k ? kBc7Anchor2[s.part] : 0;
        anchor[k] = a;
        if (!(s.sel[a] & (1u << (ib - 1)))) continue;
        for (int t = 0; t < 16; ++t)
            if ((nsub == 1 ? 0 : shape2_of(s.part, t)) == k) s.sel[t] = (uint8_t)(((1u << ib) - 1) - s.sel[t]);
        const px4 tmp = s.lo[k];
        s.lo[k] = s.hi[k];
        s.hi[k] = tmp;
        if (s.mode == 6) {   /* mode 1 shares its p-bit per subset */
            const uint32_t t = s.pb[k][0];
            s.pb[k][0] = s.pb[k][1];
            s.pb[k][1] = t;
        }
    }
    memset(out, 0, 16);
    uint32_t pos = 0;
    put_bits(out, &pos, 1u << s.mode, (uint32_t)s.mode + 1);
    if (s.mode == 1) put_bits(out, &pos, (uint32_t)s.part, 6);
    const int ncomp = s.mode == 6 ? 4 : 3;
    const uint32_t cb = s.mode == 6 ? 7 : 6;
    for (int c = 0; c < ncomp; ++c)
        for (int k = 0; k < nsub; ++k) {
            put_bits(out, &pos, s.lo[k].c[c], cb);
            put_bits(out, &pos, s.hi[k].c[c], cb);
        }
    for (int k = 0; k < nsub; ++k) {
        put_bits(out, &pos, s.pb[k][0], 1);
        if (s.mode == 6) put_bits(out, &pos, s.pb[k][1], 1);
    }
    for (int t = 0; t < 16; ++t) put_bits(out, &pos, s.sel[t], (t == anchor[0] || t == anchor[1]) ? ib - 1 : ib);
}

static float g_w3x[32], g_w4x[64];

static void init_tables(void)
{
    init_one_colour();
    for (int i = 0; i < 32; ++i) g_w3x[i] = bits_f(kEncW3x[i]);
    for (int i = 0; i < 64; ++i) g_w4x[i] = bits_f(kEncW4x[i]);
}

/* bc7enc16_compress_block :1517-1547 with handle_alpha_block / handle_opaque_block :1390-1515 */
static void bc7enc_block(const px4 px[16], const cfg_t *cfg, uint8_t out[16])
{
    int has_alpha = 0;
    for (int t = 0; t < 16; ++t) has_alpha |= px[t].c[3] < 255;
    cell_in ci;
    ci.selw = kW4, ci.selx = g_w4x, ci.nsel = 16, ci.cbits = 7;
    ci.share_pbit = 0;
    ci.perceptual = cfg->perceptual;
    ci.n = 16, ci.px = px, ci.w = cfg->w;
    ci.alpha = has_alpha;
    cell_out r6;
    const uint64_t e6 = cell(6, &ci, &r6, cfg);
    block_sol s;
    memset(&s, 0, sizeof(s));
    s.mode = 6;
    memcpy(s.sel, r6.sel, 16);
    s.lo[0] = r6.lo, s.hi[0] = r6.hi;
    s.pb[0][0] = r6.pb[0], s.pb[0][1] = r6.pb[1];
    if (!has_alpha && e6 > 0 && cfg->max_parts > 0) {
        const int part = pick_partition(px, cfg);
        px4 sub[2][16];
        uint8_t where[2][16];
        uint32_t cnt[2] = {0, 0};
        for (int t = 0; t < 16; ++t) {
            const int k = shape2_of(part, t);
            where[k][cnt[k]] = (uint8_t)t;
            sub[k][cnt[k]++] = px[t];
        }
        ci.selw = kW3, ci.selx = g_w3x, ci.nsel = 8, ci.cbits = 6, ci.share_pbit = 1;
        cell_out r1[2];
        uint64_t e1 = 0;
        for (int k = 0; k < 2; ++k) {   /* the reference stops once e1 > e6: only '<' decides */
            ci.n = cnt[k], ci.px = sub[k];
            e1 += cell(1, &ci, &r1[k], cfg);
        }
        if (e1 < e6) {
            s.mode = 1, s.part = part;
            for (int k = 0; k < 2; ++k) {
                for (uint32_t i = 0; i < cnt[k]; ++i) s.sel[where[k][i]] = r1[k].sel[i];
                s.lo[k] = r1[k].lo, s.hi[k] = r1[k].hi;
                s.pb[k][0] = r1[k].pb[0];
            }
        }
    }
    pack_block(s, out);
}

void orc_bc7enc_block(const uint8_t rgba[64], int fast, int perceptual, uint8_t out[16])
{
    cfg_t cfg;
    init_tables();
    make_cfg(fast, perceptual, &cfg);
    bc7enc_block((const px4 *)rgba, &cfg, out);
}

/* Image_CompressRichGel999BC7 :21-71 over an 8-bit source: ReadNxNBlockF (edge clamp,
 * alpha forced to 1 without an alpha channel), then TinyImageFormat_EncodeLogicalPixelsF
 * to RGBA8 -- the identity on UNORM8 texels (v/255.0f * 255 rounds back to v). */
int orc_encode_image_bc7enc(const uint8_t *src, uint32_t width, uint32_t height, uint32_t slices, uint32_t channels,
                            int fast, int perceptual, uint8_t *dst)
{
    if (!src || !dst || !width || !height || !slices || channels < 1 || channels > 4) return -1;
    cfg_t cfg;
    init_tables();
    make_cfg(fast, perceptual, &cfg);
    const uint32_t bx = (width + 3) / 4, by = (height + 3) / 4;
    for (uint32_t s = 0; s < slices; ++s) {
        const uint8_t *img = src + (size_t)width * height * channels * s;
        for (uint32_t y = 0; y < by; ++y)
            for (uint32_t x = 0; x < bx; ++x) {
                px4 px[16];
                for (int t = 0; t < 16; ++t) {
                    uint32_t sy = y * 4 + (uint32_t)(t >> 2), sx = x * 4 + (uint32_t)(t & 3);
                    sy = sy >= height ? height - 1 : sy;
                    sx = sx >= width ? width - 1 : sx;
                    const uint8_t *p = img + ((size_t)sy * width + sx) * channels;
                    px[t].c[0] = p[0];
                    px[t].c[1] = channels > 1 ? p[1] : 0;
                    px[t].c[2] = channels > 2 ? p[2] : 0;
                    px[t].c[3] = channels > 3 ? p[3] : 255;
                }
                bc7enc_block(px, &cfg, dst + (((size_t)s * by + y) * bx + x) * 16);
            }
    }
    return 0;
}

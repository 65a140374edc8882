/* Search-pruning study driver (instrumentation, not product code).
 *
 * Built together with the oracle's BC7 restatement under -DORC_TRACE
 * (tools/prune_study.py does it in /tmp): encodes each float block with
 * orc_bc7_block at default quality and records, per single-index mode and
 * shaken partition rank, the quantiser error (stored_err of the rank) and
 * the shaken error, plus every mode's final error.  Python then simulates
 * pruning policies on those arrays. */
#include <pthread.h>
#include <stdint.h>
#include <string.h>

extern void (*orc_bc7_trace)(int kind, int mode, int rank, int part, double err, const double *sub_err);
double orc_bc7_block(const float inN[64], uint8_t mode_mask, int src_has_alpha, float quality_f,
                     int colour_restrict, int alpha_restrict, float performance_f, uint8_t out[16]);

static __thread double *t_q, *t_s, *t_m, *t_all;
static __thread int *t_p;

static void cb(int kind, int mode, int rank, int part, double err, const double *sub_err)
{
    (void)sub_err;
    if (kind == 0 && rank < 8) { t_s[mode * 8 + rank] = err; t_p[mode * 8 + rank] = part; }
    if (kind == 2 && rank < 8) t_q[mode * 8 + rank] = err;
    if (kind == 1) t_m[mode] = err;
    if (kind == 4 && t_all && rank < 64) t_all[mode * 64 + rank] = err;
}

typedef struct {
    const float *blocks;
    int n, tid, nth;
    double *q, *s, *m, *best, *all;
    int *p;
    uint8_t *out;
} job;

static void *work(void *a)
{
    job *j = (job *)a;
    for (int i = j->tid; i < j->n; i += j->nth) {
        t_q = j->q + (size_t)i * 64;
        t_s = j->s + (size_t)i * 64;
        t_m = j->m + (size_t)i * 8;
        t_p = j->p + (size_t)i * 64;
        t_all = j->all ? j->all + (size_t)i * 512 : 0;
        j->best[i] = orc_bc7_block(j->blocks + (size_t)i * 64, 0xFF, 1, 1.0f, 1, 1, 1.0f, j->out + (size_t)i * 16);
    }
    return 0;
}

/* q, s: [n][8 modes][8 ranks]; m: [n][8]; p: [n][8][8] partitions; all: [n][8][64] quantiser
 * error of every partition (or NULL); unset = -1 */
int study(const float *blocks, int n, int threads, double *q, double *s, double *m, int *p, double *best, uint8_t *out,
          double *all)
{
    orc_bc7_trace = cb;
    for (size_t k = 0; k < (size_t)n * 64; ++k) { q[k] = -1; s[k] = -1; p[k] = -1; }
    for (size_t k = 0; k < (size_t)n * 8; ++k) m[k] = -1;
    if (all) for (size_t k = 0; k < (size_t)n * 512; ++k) all[k] = -1;
    pthread_t th[64];
    job jb[64];
    if (threads > 64) threads = 64;
    for (int t = 0; t < threads; ++t) {
        jb[t] = (job){blocks, n, t, threads, q, s, m, best, all, p, out};
        pthread_create(&th[t], 0, work, &jb[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(th[t], 0);
    return 0;
}

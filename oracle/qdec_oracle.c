/*
 * qdec_oracle.c -- CPU restatement of the BP(+SSF) decoding hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see qdec_oracle.h): the parity checker for the HIP
 * library and bench.py's cpu_baseline.  Never linked by exp_ldpc_amd/.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).  -ffp-contract=off
 * keeps every multiply/add separately rounded, which is what ldpc's Cython loops
 * do and what the HIP kernels are compiled to do.
 */
#include "qdec_oracle.h"

#include <math.h>
#include <omp.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int m, n;
    const int32_t* row_ptr;
    const int32_t* col_idx;
    int32_t* col_ptr;  /* n+1 */
    int32_t* col_edge; /* E: edge ids of column j in ascending row order */
    int32_t* row_of;   /* E: row of edge e */
} graph_t;

/* ------------------------------------------------------------------ BP */
#define REAL double
#define SUF f64
#define BIG 1e308
#include "bp_impl.inc"
#undef REAL
#undef SUF
#undef BIG

/* fp32 variant: ldpc has no fp32 mode; the sentinel for "min over an empty set"
 * is 1e30f (same constant as the HIP kernels). */
#define REAL float
#define SUF f32
#define BIG 1e30f
#include "bp_impl.inc"
#undef REAL
#undef SUF
#undef BIG

static int build_csc(graph_t* g) {
    const int E = g->row_ptr[g->m];
    g->col_ptr = (int32_t*)calloc((size_t)g->n + 1, sizeof(int32_t));
    g->col_edge = (int32_t*)malloc(sizeof(int32_t) * (size_t)(E > 0 ? E : 1));
    g->row_of = (int32_t*)malloc(sizeof(int32_t) * (size_t)(E > 0 ? E : 1));
    if (!g->col_ptr || !g->col_edge || !g->row_of) return -1;
    for (int i = 0; i < g->m; ++i)
        for (int e = g->row_ptr[i]; e < g->row_ptr[i + 1]; ++e) g->row_of[e] = i;
    for (int e = 0; e < E; ++e) g->col_ptr[g->col_idx[e] + 1]++;
    for (int j = 0; j < g->n; ++j) g->col_ptr[j + 1] += g->col_ptr[j];
    int32_t* fill = (int32_t*)malloc(sizeof(int32_t) * (size_t)(g->n > 0 ? g->n : 1));
    if (!fill) return -1;
    memcpy(fill, g->col_ptr, sizeof(int32_t) * (size_t)g->n);
    for (int i = 0; i < g->m; ++i) /* rows ascending -> column lists ascending in row */
        for (int e = g->row_ptr[i]; e < g->row_ptr[i + 1]; ++e) g->col_edge[fill[g->col_idx[e]]++] = e;
    free(fill);
    return 0;
}

/* ------------------------------------------------------------------ SSF
 * Spec (DESIGN.md "SSF spec"): flip sets are the non-empty subsets F of each
 * generator support (rows of gen_ptr/gen_idx, i.e. X-check rows of Hx).  One step
 * picks the (g, F) maximising gain(F)/|F| where gain(F) = |s| - |s xor H 1_F|,
 * among gain > 0; ties -> lowest g, then lowest subset bitmask (bit k <-> k-th
 * entry of row g, entries ascending).  Apply x ^= 1_F, s ^= H 1_F; repeat until no
 * positive gain or max_steps.  Brute force with cross-multiplied ratio compare. */
static int ssf_run(const graph_t* g, int32_t n_gen, const int32_t* gen_ptr, const int32_t* gen_idx,
                   uint8_t* s, uint8_t* x, int max_steps, int* touched, int* cnt) {
    int steps = 0;
    for (;;) {
        if (max_steps > 0 && steps >= max_steps) break;
        int bg = -1, bt = 0, bgain = 0, bsize = 1;
        for (int gi = 0; gi < n_gen; ++gi) {
            const int a = gen_ptr[gi], w = gen_ptr[gi + 1] - a;
            for (int t = 1; t < (1 << w); ++t) {
                int nt = 0, size = 0;
                for (int k = 0; k < w; ++k) {
                    if (!((t >> k) & 1)) continue;
                    ++size;
                    const int q = gen_idx[a + k];
                    for (int u = g->col_ptr[q]; u < g->col_ptr[q + 1]; ++u) {
                        const int c = g->row_of[g->col_edge[u]];
                        if (cnt[c] == 0) touched[nt++] = c;
                        cnt[c] ^= 2; /* bit1 toggles parity; value 0 marks untouched */
                        cnt[c] |= 1;
                    }
                }
                int gain = 0;
                for (int u = 0; u < nt; ++u) {
                    const int c = touched[u];
                    if (cnt[c] & 2) gain += s[c] ? 1 : -1;
                    cnt[c] = 0;
                }
                if (gain > 0 && (bg < 0 || (long)gain * bsize > (long)bgain * size)) {
                    bg = gi; bt = t; bgain = gain; bsize = size;
                }
            }
        }
        if (bg < 0) break;
        const int a = gen_ptr[bg], w = gen_ptr[bg + 1] - a;
        for (int k = 0; k < w; ++k) {
            if (!((bt >> k) & 1)) continue;
            const int q = gen_idx[a + k];
            x[q] ^= 1;
            for (int u = g->col_ptr[q]; u < g->col_ptr[q + 1]; ++u) s[g->row_of[g->col_edge[u]]] ^= 1;
        }
        ++steps;
    }
    return steps;
}


/* Same spec as ssf_run, evaluated with per-generator local-check bitmasks
 * (popcount of s_local ^ M_F, subsets in ascending bitmask order).  Used for the
 * timed CPU baseline; tests check it equals ssf_run bit for bit. */
typedef struct {
    int n_gen;
    int* w;          /* [n_gen] */
    int* nlc;        /* [n_gen] */
    int* lc;         /* [n_gen][32] */
    uint32_t* qm;    /* [n_gen][16] */
    const int32_t* gen_ptr;
    const int32_t* gen_idx;
} ssf_tables_t;

static int ssf_tables_build(const graph_t* g, int32_t n_gen, const int32_t* gen_ptr, const int32_t* gen_idx,
                            ssf_tables_t* T) {
    T->n_gen = n_gen;
    T->gen_ptr = gen_ptr;
    T->gen_idx = gen_idx;
    T->w = (int*)calloc((size_t)n_gen, sizeof(int));
    T->nlc = (int*)calloc((size_t)n_gen, sizeof(int));
    T->lc = (int*)calloc((size_t)n_gen * 32, sizeof(int));
    T->qm = (uint32_t*)calloc((size_t)n_gen * 16, sizeof(uint32_t));
    if (!T->w || !T->nlc || !T->lc || !T->qm) return -1;
    for (int gi = 0; gi < n_gen; ++gi) {
        const int a = gen_ptr[gi], w = gen_ptr[gi + 1] - a;
        if (w > 16) return -2;
        T->w[gi] = w;
        int* lc = T->lc + (size_t)gi * 32;
        int nlc = 0;
        for (int k = 0; k < w; ++k) {
            const int q = gen_idx[a + k];
            uint32_t mask = 0;
            for (int u = g->col_ptr[q]; u < g->col_ptr[q + 1]; ++u) {
                const int c = g->row_of[g->col_edge[u]];
                int pos = -1;
                for (int t = 0; t < nlc; ++t) if (lc[t] == c) { pos = t; break; }
                if (pos < 0) {
                    if (nlc >= 32) return -3;
                    pos = nlc;
                    lc[nlc++] = c;
                }
                mask ^= 1u << pos;
            }
            T->qm[(size_t)gi * 16 + k] = mask;
        }
        T->nlc[gi] = nlc;
    }
    return 0;
}

static void ssf_tables_free(ssf_tables_t* T) {
    free(T->w); free(T->nlc); free(T->lc); free(T->qm);
}

static int ssf_run_fast(const graph_t* g, const ssf_tables_t* T, uint8_t* s, uint8_t* x, int max_steps,
                        uint32_t* Mt) {
    int steps = 0;
    for (;;) {
        if (max_steps > 0 && steps >= max_steps) break;
        int bg = -1, bt = 0, bgain = 0, bsize = 1;
        for (int gi = 0; gi < T->n_gen; ++gi) {
            const int w = T->w[gi], nlc = T->nlc[gi];
            const int* lc = T->lc + (size_t)gi * 32;
            const uint32_t* qm = T->qm + (size_t)gi * 16;
            uint32_t sl = 0;
            for (int c = 0; c < nlc; ++c) sl |= (uint32_t)(s[lc[c]] & 1) << c;
            const int base = __builtin_popcount(sl);
            if (base == 0) continue; /* no subset can have positive gain */
            Mt[0] = 0;
            for (int t = 1; t < (1 << w); ++t) {
                Mt[t] = Mt[t & (t - 1)] ^ qm[__builtin_ctz(t)];
                const int gain = base - __builtin_popcount(sl ^ Mt[t]);
                if (gain <= 0) continue;
                const int size = __builtin_popcount(t);
                if (bg < 0 || (long)gain * bsize > (long)bgain * size) {
                    bg = gi; bt = t; bgain = gain; bsize = size;
                }
            }
        }
        if (bg < 0) break;
        const int a = T->gen_ptr[bg], w = T->gen_ptr[bg + 1] - a;
        for (int k = 0; k < w; ++k) {
            if (!((bt >> k) & 1)) continue;
            const int q = T->gen_idx[a + k];
            x[q] ^= 1;
            for (int u = g->col_ptr[q]; u < g->col_ptr[q + 1]; ++u) s[g->row_of[g->col_edge[u]]] ^= 1;
        }
        ++steps;
    }
    return steps;
}

/* ------------------------------------------------------------------ driver */
int qdo_decode_batch(int32_t m, int32_t n, const int32_t* row_ptr, const int32_t* col_idx,
                     const double* channel_probs, int32_t method, int32_t precision,
                     int32_t max_iter, double ms_scaling,
                     int32_t ssf, int32_t ssf_max_steps,
                     int32_t n_gen, const int32_t* gen_ptr, const int32_t* gen_idx,
                     int32_t n_data, int32_t fold_blocks,
                     int32_t k, const uint8_t* lz,
                     int64_t B, const uint8_t* syn, const uint8_t* base, const uint8_t* readout,
                     int32_t syn_flags,
                     uint8_t* x_out, uint8_t* corr_out, double* llr_out,
                     int32_t* iters, uint8_t* status, int32_t* ssf_steps, uint8_t* fail,
                     int32_t ssf_impl, int32_t nthreads) {
    if (m < 0 || n <= 0 || B < 0 || !row_ptr || !col_idx || !channel_probs) return -1;
    if (method != QDO_PRODUCT_SUM && method != QDO_MIN_SUM) return -2;
    if (ssf && (!gen_ptr || !gen_idx || n_gen <= 0)) return -3;
    if (n_data <= 0 || fold_blocks <= 0 || (int64_t)n_data * fold_blocks > n) return -4;
    if (max_iter <= 0) max_iter = n; /* ldpc v1: max_iter 0 -> n */

    graph_t g = {m, n, row_ptr, col_idx, NULL, NULL, NULL};
    if (build_csc(&g)) return -5;
    ssf_tables_t st;
    memset(&st, 0, sizeof(st));
    if (ssf && ssf_impl == QDO_SSF_FAST && ssf_tables_build(&g, n_gen, gen_ptr, gen_idx, &st)) {
        ssf_tables_free(&st);
        return -6;
    }
    const int E = row_ptr[m];

    double* llr64 = (double*)malloc(sizeof(double) * (size_t)n);
    float* llr32 = (float*)malloc(sizeof(float) * (size_t)n);
    for (int j = 0; j < n; ++j) {
        const double p = channel_probs[j];
        const double v = (method == QDO_MIN_SUM) ? log((1 - p) / p) : p / (1 - p);
        llr64[j] = v;
        llr32[j] = (float)v;
    }
    if (nthreads > 0) omp_set_num_threads(nthreads);
    int rc = 0;

#pragma omp parallel
    {
        double* b2c64 = (double*)malloc(sizeof(double) * (size_t)(E + 1));
        double* c2b64 = (double*)malloc(sizeof(double) * (size_t)(E + 1));
        float* b2c32 = (float*)malloc(sizeof(float) * (size_t)(E + 1));
        float* c2b32 = (float*)malloc(sizeof(float) * (size_t)(E + 1));
        int* sg = (int*)malloc(sizeof(int) * (size_t)(E + 1));
        double* lpr64 = (double*)malloc(sizeof(double) * (size_t)n);
        float* lpr32 = (float*)malloc(sizeof(float) * (size_t)n);
        uint8_t* s = (uint8_t*)malloc((size_t)m + 1);
        uint8_t* hx = (uint8_t*)malloc((size_t)m + 1);
        uint8_t* x = (uint8_t*)malloc((size_t)n);
        uint8_t* corr = (uint8_t*)malloc((size_t)n_data);
        int* touched = (int*)malloc(sizeof(int) * (size_t)(m + 1));
        int* cnt = (int*)calloc((size_t)m + 1, sizeof(int));
        uint32_t* Mt = (uint32_t*)malloc(sizeof(uint32_t) * 65536);

#pragma omp for schedule(dynamic, 64)
        for (int64_t b = 0; b < B; ++b) {
            /* 1. syndrome */
            for (int i = 0; i < m; ++i) s[i] = syn ? (syn[b * m + i] & 1) : 0;
            if (syn_flags & (QDO_SYN_ADD_BASE | QDO_SYN_ADD_READOUT)) {
                for (int i = 0; i < m; ++i) {
                    uint8_t p = 0;
                    for (int e = row_ptr[i]; e < row_ptr[i + 1]; ++e) {
                        const int j = col_idx[e];
                        if (j >= n_data) continue;
                        if ((syn_flags & QDO_SYN_ADD_BASE) && base) p ^= base[b * n_data + j] & 1;
                        if ((syn_flags & QDO_SYN_ADD_READOUT) && readout) p ^= readout[b * n_data + j] & 1;
                    }
                    s[i] ^= p;
                }
            }
            /* 2. BP */
            int it = 0, conv;
            if (precision == QDO_F32) {
                conv = (method == QDO_MIN_SUM)
                    ? bp_ms_f32(&g, llr32, max_iter, ms_scaling, s, b2c32, c2b32, sg, x, hx, lpr32, &it)
                    : bp_ps_f32(&g, llr32, max_iter, s, b2c32, c2b32, x, hx, lpr32, &it);
                if (llr_out) for (int j = 0; j < n; ++j) llr_out[b * n + j] = (double)lpr32[j];
            } else {
                conv = (method == QDO_MIN_SUM)
                    ? bp_ms_f64(&g, llr64, max_iter, ms_scaling, s, b2c64, c2b64, sg, x, hx, lpr64, &it)
                    : bp_ps_f64(&g, llr64, max_iter, s, b2c64, c2b64, x, hx, lpr64, &it);
                if (llr_out) memcpy(llr_out + b * n, lpr64, sizeof(double) * (size_t)n);
            }
            /* 3. SSF on the residual syndrome s ^ H x */
            int steps = 0, satisfied = conv;
            if (ssf && !conv) {
                for (int i = 0; i < m; ++i) hx[i] ^= s[i];
                steps = (ssf_impl == QDO_SSF_FAST)
                    ? ssf_run_fast(&g, &st, hx, x, ssf_max_steps, Mt)
                    : ssf_run(&g, n_gen, gen_ptr, gen_idx, hx, x, ssf_max_steps, touched, cnt);
                satisfied = 1;
                for (int i = 0; i < m; ++i) if (hx[i]) { satisfied = 0; break; }
            }
            /* 4. outputs */
            if (x_out) memcpy(x_out + b * n, x, (size_t)n);
            for (int q = 0; q < n_data; ++q) {
                uint8_t v = base ? (base[b * n_data + q] & 1) : 0;
                for (int t = 0; t < fold_blocks; ++t) v ^= x[t * n_data + q];
                corr[q] = v;
            }
            if (corr_out) memcpy(corr_out + b * n_data, corr, (size_t)n_data);
            if (iters) iters[b] = it;
            if (status) status[b] = (uint8_t)((conv ? QDO_ST_BP_CONVERGED : 0) | (satisfied ? QDO_ST_SATISFIED : 0));
            if (ssf_steps) ssf_steps[b] = steps;
            if (fail) {
                uint8_t f = 0;
                if (readout && lz) {
                    for (int r = 0; r < k && !f; ++r) {
                        uint8_t p = 0;
                        for (int q = 0; q < n_data; ++q)
                            p ^= (uint8_t)(lz[(int64_t)r * n_data + q] & (readout[b * n_data + q] ^ corr[q]) & 1);
                        f |= p;
                    }
                }
                fail[b] = f;
            }
        }
        free(b2c64); free(c2b64); free(b2c32); free(c2b32); free(sg); free(lpr64); free(lpr32);
        free(s); free(hx); free(x); free(corr); free(touched); free(cnt); free(Mt);
    }
    free(llr64); free(llr32);
    if (ssf && ssf_impl == QDO_SSF_FAST) ssf_tables_free(&st);
    free(g.col_ptr); free(g.col_edge); free(g.row_of);
    return rc;
}

/* ------------------------------------------------------------------ sampler */
void qdo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n1 = (uint32_t)p1;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        const uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

uint32_t qdo_threshold(double p) {
    if (!(p > 0)) return 0;
    const double v = floor(p * 4294967296.0);
    return v >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)v;
}

/* Bernoulli(thr) bits for `count` elements of event `ev` of shot `shot`, xor-ed
 * into dst. */
static void bern_xor(uint8_t* dst, int count, uint32_t thr, uint32_t ev, int64_t shot,
                     const uint32_t key[2]) {
    if (thr == 0) return;
    for (int w = 0; w * 4 < count; ++w) {
        const uint32_t ctr[4] = {(uint32_t)w, ev, (uint32_t)shot, (uint32_t)((uint64_t)shot >> 32)};
        uint32_t u[4];
        qdo_philox4x32_10(ctr, key, u);
        for (int l = 0; l < 4 && 4 * w + l < count; ++l) dst[4 * w + l] ^= (uint8_t)(u[l] < thr);
    }
}

int qdo_sample_storage(int32_t m, int32_t n, const int32_t* row_ptr, const int32_t* col_idx,
                       int32_t rounds, double p_data, double p_meas,
                       uint32_t seed, uint32_t stream, int64_t shot0, int64_t B,
                       uint8_t* syn, uint8_t* readout, int32_t nthreads) {
    if (m <= 0 || n <= 0 || rounds < 0 || B < 0 || !syn || !readout) return -1;
    const uint32_t key[2] = {seed, stream};
    /* DEPOLARIZE1(p) flips the Z-basis record with its X or Y component: 2p/3 */
    const uint32_t td = qdo_threshold(2.0 * p_data / 3.0);
    const uint32_t tm = qdo_threshold(p_meas);
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
    {
        uint8_t* cum = (uint8_t*)malloc((size_t)n);
        uint8_t* prev = (uint8_t*)malloc((size_t)m);
        uint8_t* cur = (uint8_t*)malloc((size_t)m);
#pragma omp for schedule(static)
        for (int64_t b = 0; b < B; ++b) {
            const int64_t shot = shot0 + b;
            uint8_t* out = syn + b * (int64_t)(rounds + 1) * m;
            memset(cum, 0, (size_t)n);
            memset(prev, 0, (size_t)m);
            for (int t = 0; t < rounds; ++t) {
                bern_xor(cum, n, td, 4u * t + 0u, shot, key);           /* before X-check readout */
                for (int i = 0; i < m; ++i) {                          /* Z-check outcome s_t */
                    uint8_t p = 0;
                    for (int e = row_ptr[i]; e < row_ptr[i + 1]; ++e) p ^= cum[col_idx[e]];
                    cur[i] = p;
                }
                bern_xor(cur, m, tm, 4u * t + 1u, shot, key);           /* MRX(pm) flips */
                bern_xor(cum, n, td, 4u * t + 2u, shot, key);           /* before Z-check readout */
                if (t >= 1) bern_xor(cum, n, td, 4u * t + 3u, shot, key); /* end of REPEAT body */
                for (int i = 0; i < m; ++i) { out[t * m + i] = cur[i] ^ prev[i]; prev[i] = cur[i]; }
            }
            uint8_t* rd = readout + b * (int64_t)n;
            memcpy(rd, cum, (size_t)n);
            if (rounds == 0) bern_xor(rd, n, td, 0u, shot, key);        /* single timestep: noise then MZ */
            bern_xor(rd, n, tm, rounds == 0 ? 1u : 4u * rounds, shot, key); /* MZ(pm) flips */
            for (int i = 0; i < m; ++i) {
                uint8_t p = 0;
                for (int e = row_ptr[i]; e < row_ptr[i + 1]; ++e) p ^= rd[col_idx[e]];
                out[rounds * m + i] = p ^ prev[i];
            }
        }
        free(cum); free(prev); free(cur);
    }
    return 0;
}

/* ---- OSD (bposd post-processing; the reference-default CPU leg) ---- */
#include "osd_impl.inc"

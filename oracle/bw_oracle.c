/*
 * bw_oracle.c — CPU restatement of the reference Baum-Welch path.  TEST INFRASTRUCTURE ONLY.
 *
 * This is the parity oracle for the MI355X build.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it, and only as the checker (never as the thing
 * measured or shipped).  The product path (hmm_training_amd/) never links or calls it.
 *
 * It restates, in fp64 LOG domain exactly like the reference, DemianMArin/HMM_Training
 * HMM/hmm_training.py (reference @ 2025-06-13):
 *   safe_log            :46-54      -> o_safe_log
 *   log_sum_exp         :66-79      -> lse_t (online form: drops -inf terms, max + log sum exp)
 *   calculate_log_alpha :122-160    -> inside o_forward
 *   calculate_log_beta  :163-199    -> inside o_backward
 *   hmm_training        :265-541    -> oracle_hmm_training (E-step :351-410, M-step :415-500,
 *                                      convergence :503-521, finalise :524-541)
 * and HMM/hmm_testing.py calculate_log_likelihood :49-104 -> oracle_forward_loglik.
 *
 * Pinning: tests/test_oracle_golden.py checks this file against the golden vectors that
 * tests/golden/make_golden.py produced by running the reference itself.
 *
 * The one liberty taken: log_sum_exp over a term list is evaluated as an online
 * (running max, running sum) accumulator instead of materialising the list; the result is the
 * same quantity (max + log sum exp(x - max) over the finite terms) up to fp64 rounding order.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NEG_INF (-INFINITY)

/* ---- online log-sum-exp accumulator: hmm_training.py:66-79 semantics ---------------------- */
typedef struct { double m; double s; } lse_t;

static inline void lse_init(lse_t *a) { a->m = NEG_INF; a->s = 0.0; }

static inline void lse_add(lse_t *a, double x) {
    if (x == NEG_INF) return;                /* :70-74 -inf terms are removed */
    if (a->m == NEG_INF) { a->m = x; a->s = 1.0; return; }
    if (x <= a->m) { a->s += exp(x - a->m); }
    else { a->s = a->s * exp(a->m - x) + 1.0; a->m = x; }
}

static inline int lse_any(const lse_t *a) { return a->m != NEG_INF; }

static inline double lse_value(const lse_t *a) {     /* :71-76 */
    if (a->m == NEG_INF) return NEG_INF;
    return a->m + log(a->s);
}

/* safe_log :46-54 */
static inline double o_safe_log(double x) { return x > 0.0 ? log(x) : NEG_INF; }
/* safe_exp :56-64 */
static inline double o_safe_exp(double x) { return x != NEG_INF ? exp(x) : 0.0; }

/* ---- forward pass: hmm_training.py:357-368 + calculate_log_alpha :122-160 ----------------- */
static void o_forward(const int64_t *obs, int64_t T, int N, int M, const double *lpi, const double *la,
                      const double *lb, double *alpha /* [N][T] */) {
    for (int s = 0; s < N; ++s) alpha[(int64_t)s * T + 0] = lpi[s] + lb[(int64_t)s * M + obs[0]];  /* :360 */
    for (int64_t t = 1; t < T; ++t) {
        for (int j = 0; j < N; ++j) {
            lse_t acc; lse_init(&acc);
            int any = 0;
            for (int i = 0; i < N; ++i) {                                  /* :141-147 */
                double ap = alpha[(int64_t)i * T + t - 1], a = la[i * N + j];
                if (ap != NEG_INF && a != NEG_INF) { lse_add(&acc, ap + a); any = 1; }
            }
            double out = NEG_INF;
            if (any) {                                                     /* :149-158 */
                double b = lb[(int64_t)j * M + obs[t]];
                if (b != NEG_INF) out = lse_value(&acc) + b;
            }
            alpha[(int64_t)j * T + t] = out;
        }
    }
}

/* ---- backward pass: hmm_training.py:363,371-373 + calculate_log_beta :163-199 ------------- */
static void o_backward(const int64_t *obs, int64_t T, int N, int M, const double *la, const double *lb,
                       double *beta /* [N][T] */) {
    for (int s = 0; s < N; ++s) beta[(int64_t)s * T + T - 1] = 0.0;      /* :363 */
    for (int64_t t = T - 2; t >= 0; --t) {
        int64_t o = obs[t + 1];
        for (int i = 0; i < N; ++i) {
            lse_t acc; lse_init(&acc);
            int any = 0;
            for (int j = 0; j < N; ++j) {                                  /* :182-193 */
                double a = la[i * N + j], b = lb[(int64_t)j * M + o], bn = beta[(int64_t)j * T + t + 1];
                if (a != NEG_INF && b != NEG_INF && bn != NEG_INF) { lse_add(&acc, a + b + bn); any = 1; }
            }
            beta[(int64_t)i * T + t] = any ? lse_value(&acc) : NEG_INF;     /* :195-199 */
        }
    }
}

/* LSE over alpha[:, T-1]: :376-377 */
static double o_loglik_from_alpha(const double *alpha, int64_t T, int N) {
    lse_t acc; lse_init(&acc);
    for (int s = 0; s < N; ++s) lse_add(&acc, alpha[(int64_t)s * T + T - 1]);
    return lse_value(&acc);
}

/* one sequence's terms into the accumulators (the body of :351-410 for utterance r) */
static void o_accum_seq(const int64_t *obs, int64_t T, int N, int M, const double *lpi, const double *la,
                        const double *lb, double *alpha, double *beta, lse_t *a_pi, lse_t *a_xi, lse_t *a_gex,
                        lse_t *a_gall, lse_t *a_b, double *logP_r) {
    o_forward(obs, T, N, M, lpi, la, lb, alpha);
    o_backward(obs, T, N, M, la, lb, beta);
    double lp = o_loglik_from_alpha(alpha, T, N);
    *logP_r = lp;
    if (lp == NEG_INF) return;                 /* :391-394, :401-410: gamma and xi all -inf */
    for (int64_t t = 0; t < T; ++t) {
        int64_t o = obs[t];
        for (int i = 0; i < N; ++i) {
            double g = alpha[(int64_t)i * T + t] + beta[(int64_t)i * T + t] - lp;          /* :392 */
            if (g == NEG_INF) continue;
            if (t == 0) lse_add(&a_pi[i], g);                                              /* :420 */
            if (t < T - 1) lse_add(&a_gex[i], g);                                          /* :436 */
            lse_add(&a_gall[i], g);                                                        /* :467 */
            lse_add(&a_b[(int64_t)i * M + o], g);                                          /* :483 */
        }
        if (t < T - 1) {
            int64_t on = obs[t + 1];
            for (int i = 0; i < N; ++i)
                for (int j = 0; j < N; ++j) {                                              /* :402-408 */
                    double x = alpha[(int64_t)i * T + t] + la[i * N + j] + lb[(int64_t)j * M + on] +
                               beta[(int64_t)j * T + t + 1] - lp;
                    lse_add(&a_xi[i * N + j], x);
                }
        }
    }
}

/* merge two online accumulators (the LSE of the union of their term lists) */
static inline void lse_merge(lse_t *a, const lse_t *b) {
    if (b->m == NEG_INF) return;
    if (a->m == NEG_INF) { *a = *b; return; }
    if (b->m <= a->m) a->s += b->s * exp(b->m - a->m);
    else { a->s = a->s * exp(a->m - b->m) + b->s; a->m = b->m; }
}

/* Threads used by oracle_estep_logstats (and so oracle_hmm_training): 1 = the serial restatement
 * the parity tests use.  bench.py's cpu_baseline leg sets the host's core count (OpenMP over
 * utterances, per-thread accumulators merged in thread order: same terms, different rounding order). */
static int g_threads = 1;
int oracle_set_threads(int n) {
#ifdef _OPENMP
    g_threads = n > 0 ? n : 1;
#else
    (void)n;
    g_threads = 1;
#endif
    return g_threads;
}

/*
 * E-step sufficient statistics in the log domain (hmm_training.py:351-410 feeding :415-500):
 *   lpi_num[N]    = LSE_r gamma_0^r(i)                       (:415-424, before "- log R")
 *   lxi[N*N]      = LSE_{r,t<T-1} xi_t^r(i,j)                (:443-455 numerator)
 *   lgden_ex[N]   = LSE_{r,t<=T-2} gamma_t^r(i)              (:431-441 denominator)
 *   lgden_all[N]  = LSE_{r,t} gamma_t^r(j)                   (:462-472 denominator)
 *   lbnum[N*M]    = LSE_{r,t:o_t=k} gamma_t^r(j)             (:474-495 numerator; -inf if none)
 *   logP[R]                                                  (:375-377)
 * Returns 0, or -1 on allocation failure, -2 on an empty sequence (the reference raises
 * IndexError at :376 for T=0).
 */
int oracle_estep_logstats(const int64_t *offsets, const int64_t *symbols, int64_t R, int N, int M,
                          const double *lpi, const double *la, const double *lb,
                          double *lpi_num, double *lxi, double *lgden_ex, double *lgden_all, double *lbnum,
                          double *logP) {
    int64_t Tmax = 0;
    for (int64_t r = 0; r < R; ++r) {
        int64_t T = offsets[r + 1] - offsets[r];
        if (T <= 0) return -2;
        if (T > Tmax) Tmax = T;
    }
    int nth = g_threads;
    if (R < nth) nth = R > 0 ? (int)R : 1;
    /* per thread: N + N*N + N + N + N*M accumulators */
    const size_t nacc = (size_t)N * (3 + N) + (size_t)N * M;
    lse_t *acc = (lse_t *)malloc(sizeof(lse_t) * nacc * nth);
    if (!acc) return -1;
    for (size_t i = 0; i < nacc * nth; ++i) lse_init(&acc[i]);
    int fail = 0;
#ifdef _OPENMP
#pragma omp parallel num_threads(nth) reduction(| : fail)
#endif
    {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        lse_t *a_pi = acc + nacc * tid, *a_xi = a_pi + N, *a_gex = a_xi + N * N, *a_gall = a_gex + N;
        lse_t *a_b = a_gall + N;
        double *alpha = (double *)malloc(sizeof(double) * (size_t)N * (size_t)(Tmax ? Tmax : 1));
        double *beta = (double *)malloc(sizeof(double) * (size_t)N * (size_t)(Tmax ? Tmax : 1));
        if (!alpha || !beta) {
            fail = 1;
        } else {
            /* contiguous blocks of utterances per thread (static schedule): a fixed merge order */
            int64_t lo = R * tid / nth, hi = R * (tid + 1) / nth;
            for (int64_t r = lo; r < hi; ++r)
                o_accum_seq(symbols + offsets[r], offsets[r + 1] - offsets[r], N, M, lpi, la, lb, alpha, beta,
                            a_pi, a_xi, a_gex, a_gall, a_b, &logP[r]);
        }
        free(alpha);
        free(beta);
    }
    if (fail) { free(acc); return -1; }
    for (int th = 1; th < nth; ++th)
        for (size_t i = 0; i < nacc; ++i) lse_merge(&acc[i], &acc[nacc * th + i]);
    const lse_t *a_pi = acc, *a_xi = a_pi + N, *a_gex = a_xi + N * N, *a_gall = a_gex + N, *a_b = a_gall + N;
    for (int i = 0; i < N; ++i) {
        lpi_num[i] = lse_value(&a_pi[i]);
        lgden_ex[i] = lse_value(&a_gex[i]);
        lgden_all[i] = lse_value(&a_gall[i]);
    }
    for (int i = 0; i < N * N; ++i) lxi[i] = lse_value(&a_xi[i]);
    for (int64_t i = 0; i < (int64_t)N * M; ++i) lbnum[i] = lse_value(&a_b[i]);
    free(acc);
    return 0;
}

/* M-step from log statistics: hmm_training.py:415-500 (R counts every sequence, :424). */
void oracle_mstep_log(int64_t R, int N, int M, const double *lpi_num, const double *lxi, const double *lgden_ex,
                      const double *lgden_all, const double *lbnum, double *lpi, double *la, double *lb) {
    for (int i = 0; i < N; ++i)                                                            /* :415-424 */
        lpi[i] = lpi_num[i] != NEG_INF ? lpi_num[i] - log((double)R) : NEG_INF;
    for (int i = 0; i < N; ++i)                                                            /* :429-455 */
        for (int j = 0; j < N; ++j)
            la[i * N + j] = (lgden_ex[i] != NEG_INF && lxi[i * N + j] != NEG_INF) ? lxi[i * N + j] - lgden_ex[i]
                                                                                   : NEG_INF;
    const double floor_log = log(1e-20);                                                  /* :497 */
    for (int j = 0; j < N; ++j)                                                            /* :460-497 */
        for (int k = 0; k < M; ++k) {
            double v = NEG_INF;
            if (lgden_all[j] != NEG_INF) v = lbnum[(int64_t)j * M + k] != NEG_INF ? lbnum[(int64_t)j * M + k] - lgden_all[j]
                                                                                  : floor_log;
            lb[(int64_t)j * M + k] = v;
        }
}

/* LSE over logP: :503 */
double oracle_lse(const double *x, int64_t n) {
    lse_t acc; lse_init(&acc);
    for (int64_t i = 0; i < n; ++i) lse_add(&acc, x[i]);
    return lse_value(&acc);
}

/*
 * hmm_training :265-541 from linear initial parameters (the reference's safe_log at :323-325).
 * trace_L/trace_diff must hold max_iterations entries.  Outputs: the returned (A, B, pi)
 * (normalised, :524-541), the final unnormalised log params, and logP of the last iteration.
 * Returns the iteration count (>= 0) or a negative error.
 */
int64_t oracle_hmm_training(const int64_t *offsets, const int64_t *symbols, int64_t R, int N, int M, double epsilon,
                            int64_t max_iterations, const double *pi0, const double *A0, const double *B0,
                            double *out_A, double *out_B, double *out_pi, double *trace_L, double *trace_diff,
                            double *last_logP, double *out_lpi, double *out_la, double *out_lb) {
    size_t NN = (size_t)N * N, NM = (size_t)N * M;
    double *lpi = (double *)malloc(sizeof(double) * N), *la = (double *)malloc(sizeof(double) * NN);
    double *lb = (double *)malloc(sizeof(double) * NM);
    double *s_pi = (double *)malloc(sizeof(double) * N), *s_xi = (double *)malloc(sizeof(double) * NN);
    double *s_gex = (double *)malloc(sizeof(double) * N), *s_gall = (double *)malloc(sizeof(double) * N);
    double *s_b = (double *)malloc(sizeof(double) * NM);
    double *logP = (double *)malloc(sizeof(double) * (size_t)(R > 0 ? R : 1));
    int64_t it = 0;
    if (!lpi || !la || !lb || !s_pi || !s_xi || !s_gex || !s_gall || !s_b || !logP) { it = -1; goto done; }
    for (int i = 0; i < N; ++i) lpi[i] = o_safe_log(pi0[i]);                              /* :323-325 */
    for (size_t i = 0; i < NN; ++i) la[i] = o_safe_log(A0[i]);
    for (size_t i = 0; i < NM; ++i) lb[i] = o_safe_log(B0[i]);
    for (int64_t r = 0; r < R; ++r) logP[r] = NEG_INF;                                     /* :332 */

    double prev = NEG_INF, diff = epsilon + 10.0;                                          /* :342-343 */
    while (diff >= epsilon && it < max_iterations) {                                       /* :346 */
        int rc = oracle_estep_logstats(offsets, symbols, R, N, M, lpi, la, lb, s_pi, s_xi, s_gex, s_gall, s_b, logP);
        if (rc != 0) { it = rc == -2 ? -2 : -1; goto done; }
        oracle_mstep_log(R, N, M, s_pi, s_xi, s_gex, s_gall, s_b, lpi, la, lb);
        double cur = oracle_lse(logP, R);                                                  /* :503 */
        diff = (prev != NEG_INF) ? fabs(cur - prev) : INFINITY;                            /* :505-508 */
        trace_L[it] = cur;
        trace_diff[it] = diff;
        prev = cur;
        it += 1;
    }
    /* finalise :524-541 */
    double ps = 0.0;
    for (int i = 0; i < N; ++i) { out_pi[i] = o_safe_exp(lpi[i]); ps += out_pi[i]; }
    for (int i = 0; i < N; ++i) out_pi[i] = out_pi[i] / ps;
    for (int i = 0; i < N; ++i) {
        double s = 0.0;
        for (int j = 0; j < N; ++j) { out_A[i * N + j] = o_safe_exp(la[i * N + j]); s += out_A[i * N + j]; }
        if (s > 0) for (int j = 0; j < N; ++j) out_A[i * N + j] /= s;
    }
    for (int i = 0; i < N; ++i) {
        double s = 0.0;
        for (int k = 0; k < M; ++k) { out_B[(size_t)i * M + k] = o_safe_exp(lb[(size_t)i * M + k]); s += out_B[(size_t)i * M + k]; }
        if (s > 0) for (int k = 0; k < M; ++k) out_B[(size_t)i * M + k] /= s;
    }
    if (last_logP) memcpy(last_logP, logP, sizeof(double) * (size_t)R);
    if (out_lpi) memcpy(out_lpi, lpi, sizeof(double) * N);
    if (out_la) memcpy(out_la, la, sizeof(double) * NN);
    if (out_lb) memcpy(out_lb, lb, sizeof(double) * NM);
done:
    free(lpi); free(la); free(lb); free(s_pi); free(s_xi); free(s_gex); free(s_gall); free(s_b); free(logP);
    return it;
}

/* hmm_testing.py:49-104 calculate_log_likelihood: forward-only score under a LINEAR model. */
int oracle_forward_loglik(const int64_t *offsets, const int64_t *symbols, int64_t R, int N, int M, const double *pi,
                          const double *A, const double *B, double *out) {
    size_t NN = (size_t)N * N, NM = (size_t)N * M;
    int64_t Tmax = 1;
    for (int64_t r = 0; r < R; ++r) {
        int64_t T = offsets[r + 1] - offsets[r];
        if (T <= 0) return -2;                       /* :75 indexes obs[0]: IndexError on T=0 */
        if (T > Tmax) Tmax = T;
    }
    double *lpi = (double *)malloc(sizeof(double) * N), *la = (double *)malloc(sizeof(double) * NN);
    double *lb = (double *)malloc(sizeof(double) * NM), *alpha = (double *)malloc(sizeof(double) * N * (size_t)Tmax);
    if (!lpi || !la || !lb || !alpha) { free(lpi); free(la); free(lb); free(alpha); return -1; }
    for (int i = 0; i < N; ++i) lpi[i] = o_safe_log(pi[i]);                               /* :67-69 */
    for (size_t i = 0; i < NN; ++i) la[i] = o_safe_log(A[i]);
    for (size_t i = 0; i < NM; ++i) lb[i] = o_safe_log(B[i]);
    for (int64_t r = 0; r < R; ++r) {
        const int64_t *obs = symbols + offsets[r];
        int64_t T = offsets[r + 1] - offsets[r];
        /* :76-80: -inf unless both finite (same value as lpi + lb under IEEE) */
        for (int s = 0; s < N; ++s) {
            double b = lb[(size_t)s * M + obs[0]];
            alpha[(size_t)s * T] = (lpi[s] != NEG_INF && b != NEG_INF) ? lpi[s] + b : NEG_INF;
        }
        /* :87-90 reuse calculate_log_alpha */
        for (int64_t t = 1; t < T; ++t)
            for (int j = 0; j < N; ++j) {
                lse_t acc; lse_init(&acc);
                int any = 0;
                for (int i = 0; i < N; ++i) {
                    double ap = alpha[(size_t)i * T + t - 1], a = la[i * N + j];
                    if (ap != NEG_INF && a != NEG_INF) { lse_add(&acc, ap + a); any = 1; }
                }
                double v = NEG_INF;
                if (any) { double b = lb[(size_t)j * M + obs[t]]; if (b != NEG_INF) v = lse_value(&acc) + b; }
                alpha[(size_t)j * T + t] = v;
            }
        out[r] = o_loglik_from_alpha(alpha, T, N);                                         /* :94-102 */
    }
    free(lpi); free(la); free(lb); free(alpha);
    return 0;
}

/* hmm_training.py:82-120 get_observations: nearest centroid by Euclidean distance over
 * mfcc[1:], first minimum wins (strict '<' at :112). frames [F][D], centroids [K][D]. */
void oracle_vq(const double *frames, int64_t F, const double *centroids, int64_t K, int D, int64_t *out,
               double *dist_out) {
    /* hmm_training.py:94-114.  distance = np.linalg.norm(frame[1:] - centroid[1:]) (:109) =
     * sqrt(x.dot(x)); OpenBLAS ddot on these 12-element vectors is a sequential fused multiply-add
     * from element 0 (measured bit-exact against numpy here: tests/test_oracle_golden.py).  First
     * minimum wins (strict '<', :111); NaN distances never win, so the index stays 0. */
    for (int64_t f = 0; f < F; ++f) {
        double best = INFINITY;
        int64_t arg = 0;
        for (int64_t k = 0; k < K; ++k) {
            double s = 0.0;
            for (int d = 1; d < D; ++d) {
                const double e = frames[f * D + d] - centroids[k * D + d];
                s = fma(e, e, s);
            }
            const double dist = sqrt(s);
            if (dist < best) { best = dist; arg = k; }
        }
        out[f] = arg;
        if (dist_out) dist_out[f] = best;
    }
}

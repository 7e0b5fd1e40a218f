/*
 * asan_main.c — drives every entry point of bw_oracle.c under AddressSanitizer + UBSan.
 * TEST INFRASTRUCTURE ONLY (built by oracle/build_oracle.py:build_asan, run by
 * tests/test_oracle_golden.py).  Exercises: ragged lengths incl. T=1, an impossible sequence
 * (log P = -inf, hmm_training.py:391-394), empty B rows (the :497 floor / -inf rows), N=1, the
 * T=0 error return (:376), the OpenMP path with more threads than sequences, and the VQ search.
 * Prints one line per case and "asan ok" at the end; any sanitizer report aborts with non-zero.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

int64_t oracle_hmm_training(const int64_t *, const int64_t *, int64_t, int, int, double, int64_t, const double *,
                            const double *, const double *, double *, double *, double *, double *, double *,
                            double *, double *, double *, double *);
int oracle_forward_loglik(const int64_t *, const int64_t *, int64_t, int, int, const double *, const double *,
                          const double *, double *);
void oracle_vq(const double *, int64_t, const double *, int64_t, int, int64_t *, double *);
int oracle_set_threads(int);

static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static uint64_t next_u64(void) {
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return g_rng;
}
static double unif(void) { return (double)(next_u64() >> 11) / 9007199254740992.0; }

/* random row-stochastic matrix; `lr` keeps only a_ii, a_i,i+1 */
static void stochastic(double *P, int rows, int cols, int lr, int zero_col) {
    for (int i = 0; i < rows; ++i) {
        double s = 0.0;
        for (int j = 0; j < cols; ++j) {
            double v = 0.05 + unif();
            if (lr && j != i && j != i + 1) v = 0.0;
            if (j == zero_col) v = 0.0;
            P[(size_t)i * cols + j] = v;
            s += v;
        }
        for (int j = 0; j < cols; ++j) P[(size_t)i * cols + j] /= s;
    }
}

static int run_case(const char *name, int N, int M, int64_t R, int Tmax, int lr, int zero_col, int threads) {
    int64_t *off = malloc(sizeof(int64_t) * (size_t)(R + 1));
    off[0] = 0;
    for (int64_t r = 0; r < R; ++r) off[r + 1] = off[r] + 1 + (int64_t)(next_u64() % (uint64_t)Tmax);
    int64_t tot = off[R];
    int64_t *sym = malloc(sizeof(int64_t) * (size_t)(tot ? tot : 1));
    for (int64_t i = 0; i < tot; ++i) sym[i] = (int64_t)(next_u64() % (uint64_t)M);
    if (zero_col >= 0 && tot > 0) sym[0] = zero_col; /* sequence 0 impossible: log P = -inf */
    double *pi = malloc(sizeof(double) * N), *A = malloc(sizeof(double) * N * N), *B = malloc(sizeof(double) * N * M);
    stochastic(pi, 1, N, 0, -1);
    stochastic(A, N, N, lr, -1);
    stochastic(B, N, M, 0, zero_col);
    const int64_t iters = 3;
    double *oA = malloc(sizeof(double) * N * N), *oB = malloc(sizeof(double) * N * M), *opi = malloc(sizeof(double) * N);
    double *tL = malloc(sizeof(double) * iters), *tD = malloc(sizeof(double) * iters);
    double *lp = malloc(sizeof(double) * (size_t)(R ? R : 1)), *lpi = malloc(sizeof(double) * N);
    double *la = malloc(sizeof(double) * N * N), *lb = malloc(sizeof(double) * N * M);
    double *sc = malloc(sizeof(double) * (size_t)(R ? R : 1));
    oracle_set_threads(threads);
    int64_t it = oracle_hmm_training(off, sym, R, N, M, 1e-6, iters, pi, A, B, oA, oB, opi, tL, tD, lp, lpi, la, lb);
    int rc = oracle_forward_loglik(off, sym, R, N, M, opi, oA, oB, sc);
    oracle_set_threads(1);
    printf("%s: iterations=%lld L=%.6f score_rc=%d\n", name, (long long)it, it > 0 ? tL[it - 1] : NAN, rc);
    int bad = (it <= 0) || rc != 0;
    free(off); free(sym); free(pi); free(A); free(B); free(oA); free(oB); free(opi); free(tL); free(tD);
    free(lp); free(lpi); free(la); free(lb); free(sc);
    return bad;
}

int main(void) {
    int bad = 0;
    bad |= run_case("n4_k16_ragged", 4, 16, 9, 40, 1, -1, 1);
    bad |= run_case("n8_k256_lr_threads", 8, 256, 50, 120, 1, -1, 4);
    bad |= run_case("n5_dense_zero_col", 5, 32, 12, 30, 0, 7, 3);
    bad |= run_case("n1_k8", 1, 8, 6, 10, 0, -1, 1);
    bad |= run_case("n3_more_threads_than_seqs", 3, 8, 2, 5, 0, -1, 8);
    bad |= run_case("n16_t1", 16, 64, 7, 1, 0, -1, 2);
    /* T = 0 -> the error return, no out-of-bounds read */
    {
        int64_t off[3] = {0, 2, 2}, sym[2] = {1, 2};
        double pi[2] = {0.5, 0.5}, A[4] = {0.5, 0.5, 0.5, 0.5}, B[8] = {0.25, 0.25, 0.25, 0.25, 0.25, 0.25, 0.25, 0.25};
        double oA[4], oB[8], opi[2], tL[2], tD[2], lp[2], lpi[2], la[4], lb[8], sc[2];
        int64_t it = oracle_hmm_training(off, sym, 2, 2, 4, 1e-6, 2, pi, A, B, oA, oB, opi, tL, tD, lp, lpi, la, lb);
        int rc = oracle_forward_loglik(off, sym, 2, 2, 4, pi, A, B, sc);
        printf("empty_sequence: it=%lld rc=%d\n", (long long)it, rc);
        bad |= !(it == -2 && rc == -2);
    }
    /* VQ: 13-dim frames (power + 12 MFCC) against 64 centroids */
    {
        const int F = 300, K = 64, D = 13;
        double *fr = malloc(sizeof(double) * F * D), *ce = malloc(sizeof(double) * K * D), *dist = malloc(sizeof(double) * F);
        int64_t *idx = malloc(sizeof(int64_t) * F);
        for (int i = 0; i < F * D; ++i) fr[i] = unif() * 20.0 - 10.0;
        for (int i = 0; i < K * D; ++i) ce[i] = unif() * 20.0 - 10.0;
        oracle_vq(fr, F, ce, K, D, idx, dist);
        int ok = 1;
        for (int f = 0; f < F; ++f) ok &= idx[f] >= 0 && idx[f] < K && dist[f] >= 0.0;
        printf("vq: ok=%d\n", ok);
        bad |= !ok;
        free(fr); free(ce); free(dist); free(idx);
    }
    if (bad) {
        printf("asan FAILED\n");
        return 1;
    }
    printf("asan ok\n");
    return 0;
}

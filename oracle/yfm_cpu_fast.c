/*
 * yfm_cpu_fast.c — an OPTIMISED CPU implementation of the same log-likelihood, for the
 * bench's honest CPU baseline (bench.py `cpu_baseline.optimised`).  NOT the reference's
 * algorithm: it is the CPU counterpart of what the HIP kernels do, so the GPU/CPU ratio
 * measures hardware rather than the O(N³) → O(NM + M³) change of algorithm.
 *
 * TEST INFRASTRUCTURE / BASELINE ONLY: only bench.py's cpu_baseline leg and tests/ load it.
 *
 *   fixed loadings (DNS, GNS5): the collapsed form of DESIGN.md §3.1 — with G = Z'Z and
 *     R = σ²G⁻¹ fixed per candidate, each step needs z̃ = Z'ỹ_t (2N(M−1) flops) and an M×M
 *     update (LDLᵀ of P + R) — evaluated for 8 candidates at a time in structure-of-arrays
 *     form so the compiler vectorises every operation across candidates (AVX-512 / AVX2),
 *     OpenMP over blocks of candidates;
 *   TVλ EKF: the capacitance form (B̃ = σ²I + PG, 4×4 pivoted LU), one candidate per thread,
 *     exp(−λm_i) per maturity.
 * Same reference semantics as oracle/yfm_oracle.c (filter.jl:1-10, :12-80, :125-209): t = 1 not
 * accumulated, last column unused, NaN columns re-add the stale term, det < 0 → −Inf, a
 * non-finite loglik → −Inf, NaN where initialize_filter would throw.  Checked against the
 * dense oracle in tests/test_oracle.py.
 *
 * Build: gcc -O3 -march=native -fopenmp -shared -fPIC yfm_cpu_fast.c -o libyfm_cpu_fast.so -lm
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define KIND_DNS 0
#define KIND_TVL 1
#define KIND_GNS 2
#define MMAX 5
#define V 8 /* candidates per vector block */

static int state_dim(int kind) { return kind == KIND_DNS ? 3 : kind == KIND_TVL ? 4 : 5; }
static int n_lead(int kind) { return kind == KIND_DNS ? 1 : kind == KIND_TVL ? 0 : 2; }
static int param_count(int kind) {
    int M = state_dim(kind);
    return n_lead(kind) + 1 + M * (M + 1) / 2 + M + M * M;
}

/* ---------------- per-candidate setup (scalar) ---------------- */
typedef struct {
    double sig2, gam[2], Q[MMAX][MMAX], delta[MMAX], Phi[MMAX][MMAX];
} params_t;

static void decode(int kind, const double* th, int space, params_t* p) {
    int M = state_dim(kind), L = n_lead(kind), k = 0;
    for (int l = 0; l < L; ++l) p->gam[l] = th[k++];
    p->sig2 = space == 0 ? exp(th[k]) : th[k];
    ++k;
    double U[MMAX][MMAX] = {{0}};
    for (int j = 0; j < M; ++j)
        for (int i = 0; i <= j; ++i) {
            double x = th[k++];
            U[i][j] = (i == j && space == 0) ? exp(x) : x;
        }
    for (int i = 0; i < M; ++i)
        for (int j = 0; j < M; ++j) {
            double s = 0;
            for (int l = 0; l < M; ++l) s += U[l][i] * U[l][j];
            p->Q[i][j] = s;
        }
    for (int i = 0; i < M; ++i) p->delta[i] = th[k++];
    for (int i = 0; i < M; ++i)
        for (int j = 0; j < M; ++j) {
            double x = th[k++];
            if (i == j && space == 0) { double y = exp(x); x = 2.0 * y / (1.0 + y) - 1.0; }
            p->Phi[i][j] = x;
        }
}

/* Gaussian elimination with partial pivoting, row-major n×n with r right-hand sides;
 * returns 0 on an exact zero pivot, else the determinant. */
static double gauss(double* A, int n, double* X, int r) {
    double det = 1;
    for (int k = 0; k < n; ++k) {
        int p = k;
        for (int i = k + 1; i < n; ++i) if (fabs(A[i * n + k]) > fabs(A[p * n + k])) p = i;
        if (A[p * n + k] == 0.0) return 0.0;
        if (p != k) {
            det = -det;
            for (int c = 0; c < n; ++c) { double t = A[k * n + c]; A[k * n + c] = A[p * n + c]; A[p * n + c] = t; }
            for (int c = 0; c < r; ++c) { double t = X[k * r + c]; X[k * r + c] = X[p * r + c]; X[p * r + c] = t; }
        }
        det *= A[k * n + k];
        for (int i = k + 1; i < n; ++i) {
            double l = A[i * n + k] / A[k * n + k];
            for (int c = k + 1; c < n; ++c) A[i * n + c] -= l * A[k * n + c];
            for (int c = 0; c < r; ++c) X[i * r + c] -= l * X[k * r + c];
        }
    }
    for (int k = n - 1; k >= 0; --k)
        for (int c = 0; c < r; ++c) {
            double s = X[k * r + c];
            for (int j = k + 1; j < n; ++j) s -= A[k * n + j] * X[j * r + c];
            X[k * r + c] = s / A[k * n + k];
        }
    return det;
}

/* initialize_filter (filter.jl:1-10) on the symmetric subspace; 0 where the reference throws */
static int init_state(int M, const params_t* p, double* beta, double P[MMAX][MMAX]) {
    double A[MMAX * MMAX], b[MMAX];
    for (int i = 0; i < M; ++i) {
        for (int j = 0; j < M; ++j) A[i * M + j] = (i == j) - p->Phi[i][j];
        b[i] = p->delta[i];
    }
    if (gauss(A, M, b, 1) == 0.0) return 0;
    for (int i = 0; i < M; ++i) beta[i] = b[i];
    int S = M * (M + 1) / 2, r = 0;
    double L[15 * 15], q[15];
    for (int i = 0; i < M; ++i)
        for (int j = i; j < M; ++j, ++r) {
            int c = 0;
            for (int k = 0; k < M; ++k)
                for (int l = k; l < M; ++l, ++c) {
                    double s = p->Phi[i][k] * p->Phi[j][l];
                    if (k != l) s += p->Phi[i][l] * p->Phi[j][k];
                    L[r * S + c] = (r == c) - s;
                }
            q[r] = p->Q[i][j];
        }
    if (gauss(L, S, q, 1) == 0.0) return 0;
    r = 0;
    for (int i = 0; i < M; ++i)
        for (int j = i; j < M; ++j, ++r) P[i][j] = P[j][i] = q[r];
    return 1;
}

/* ---------------- fixed loadings: 8 candidates per block, collapsed form ---------------- */
typedef double vd __attribute__((vector_size(8 * V)));
typedef long long vl __attribute__((vector_size(8 * V)));
static inline vd vzero(void) { return (vd){0}; }
static inline vd vset(double x) { return (vd){0} + x; }
static inline vd vsel(vl m, vd a, vd b) { return (vd)(((vl)a & m) | ((vl)b & ~m)); }
static inline vd vabs(vd x) { return (vd)((vl)x & 0x7fffffffffffffffLL); }
#define LANE(x, v) (((double*)&(x))[v])

typedef struct {
    vd beta[MMAX], P[MMAX][MMAX], R[MMAX][MMAX], Phi[MMAX][MMAX], Q[MMAX][MMAX], delta[MMAX];
    vd rs2, sumq, mant, last_det, last_q, per_term;
    vl neg;
    int expo[V], nobs[V];
} block_t;

static void renorm(block_t* s) {
    for (int v = 0; v < V; ++v) {
        int e;
        LANE(s->mant, v) = frexp(LANE(s->mant, v), &e);
        s->expo[v] += e;
    }
}

#define FZ_M 3
#define FZ_NAME(f) f##_3
#include "yfm_cpu_fast_body.h"
#undef FZ_M
#undef FZ_NAME
#define FZ_M 5
#define FZ_NAME(f) f##_5
#include "yfm_cpu_fast_body.h"
#undef FZ_M
#undef FZ_NAME

/* Falls back to the capacitance form for candidates with ill-conditioned Z'Z (κ₁ ≥ 1e8) — the
 * same switch as the HIP kernel — one candidate at a time. */
static double capacitance_one(int kind, const params_t* p, const double* Z, const double* Y, int N, int nobs);

static void fixedz_block(int kind, const double* Y, const double* Yc, const double* ybar, const double* ytt,
                         const unsigned char* isnan_col, int N, int T, const double* mats, const double* theta,
                         int space, int b0, int nb, const int* T_use, double* out) {
    const int M = state_dim(kind), NZ = M - 1, Pk = param_count(kind);
    block_t s;
    memset(&s, 0, sizeof s);
    s.mant = vset(1.0);
    vd* Zc = aligned_alloc(64, sizeof(vd) * (size_t)NZ * N); /* [j][i], 8 candidates per vd */
    memset(Zc, 0, sizeof(vd) * (size_t)NZ * N);
    double* Zfull = malloc(sizeof(double) * (size_t)N * M);
    int active[V] = {0};
    int nmax = 0;
    for (int v = 0; v < nb; ++v) {
        const int b = b0 + v;
        params_t p;
        decode(kind, theta + (size_t)b * Pk, space, &p);
        s.nobs[v] = T_use ? T_use[b] : T;
        for (int l = 0; l < n_lead(kind); ++l) {
            double lam = 1e-2 + exp(p.gam[l]);
            for (int i = 0; i < N; ++i) {
                double tau = lam * mats[i], z = exp(-tau), sl = (1.0 - z) / tau;
                LANE(Zc[(size_t)(2 * l) * N + i], v) = sl;
                LANE(Zc[(size_t)(2 * l + 1) * N + i], v) = sl - z;
            }
        }
        /* G = Z'Z, R = σ²G⁻¹, κ₁ check, log det G */
        double G[MMAX * MMAX], X[MMAX * MMAX];
        for (int i = 0; i < N; ++i) {
            Zfull[i * M] = 1.0;
            for (int j = 0; j < NZ; ++j) Zfull[i * M + 1 + j] = LANE(Zc[(size_t)j * N + i], v);
        }
        for (int a2 = 0; a2 < M; ++a2)
            for (int c = 0; c < M; ++c) {
                double x = 0;
                for (int i = 0; i < N; ++i) x += Zfull[i * M + a2] * Zfull[i * M + c];
                G[a2 * M + c] = x;
                X[a2 * M + c] = a2 == c;
            }
        double Gc[MMAX * MMAX];
        memcpy(Gc, G, sizeof Gc);
        double detG = gauss(Gc, M, X, M);
        double nG = 0, nX = 0;
        for (int c = 0; c < M; ++c) {
            double cg = 0, cx = 0;
            for (int a2 = 0; a2 < M; ++a2) { cg += fabs(G[a2 * M + c]); cx += fabs(X[a2 * M + c]); }
            nG = fmax(nG, cg);
            nX = fmax(nX, cx);
        }
        const int collapsed = detG != 0.0 && N >= M && nG * nX < 1e8;
        double beta[MMAX], P[MMAX][MMAX];
        const int ok = init_state(M, &p, beta, P);
        if (!ok) { out[b] = NAN; continue; }
        if (!collapsed) { /* rare: this candidate alone in the capacitance form */
            out[b] = capacitance_one(kind, &p, Zfull, Y, N, s.nobs[v]);
            continue;
        }
        active[v] = 1;
        for (int a2 = 0; a2 < M; ++a2) {
            LANE(s.beta[a2], v) = beta[a2];
            LANE(s.delta[a2], v) = p.delta[a2];
            for (int c = 0; c < M; ++c) {
                LANE(s.P[a2][c], v) = P[a2][c];
                LANE(s.R[a2][c], v) = p.sig2 * 0.5 * (X[a2 * M + c] + X[c * M + a2]);
                LANE(s.Phi[a2][c], v) = p.Phi[a2][c];
                LANE(s.Q[a2][c], v) = p.Q[a2][c];
            }
        }
        LANE(s.rs2, v) = 1.0 / p.sig2;
        LANE(s.per_term, v) = (N - M) * log(p.sig2) + log(fabs(detG)) + N * log(2.0 * M_PI);
        if (s.nobs[v] > nmax) nmax = s.nobs[v];
    }
    vd zt[MMAX];
    for (int t = 0; t < nmax - 1; ++t) {
        vl upd = {0};
        for (int v = 0; v < V; ++v) upd[v] = (active[v] && t < s.nobs[v] - 1) ? -1 : 0;
        const vl accm = (vl){0} + (t >= 1 ? -1LL : 0LL);
        if (isnan_col[t]) {
            if (M == 3) predict_block_3(&s, upd, accm);
            else predict_block_5(&s, upd, accm);
        } else {
            const double* yc = Yc + (size_t)t * N;
            for (int j = 0; j < NZ; ++j) {
                const vd* Zj = Zc + (size_t)j * N;
                vd acc = vzero();
                for (int i = 0; i < N; ++i) acc += Zj[i] * yc[i];
                zt[j + 1] = acc;
            }
            if (M == 3) collapsed_step_3(&s, zt, ybar[t], ytt[t], upd, accm);
            else collapsed_step_5(&s, zt, ybar[t], ytt[t], upd, accm);
        }
        if ((t & 15) == 15) renorm(&s);
    }
    renorm(&s);
    for (int v = 0; v < nb; ++v) {
        if (!active[v]) continue;
        const int nterms = s.nobs[v] - 2 > 0 ? s.nobs[v] - 2 : 0;
        double ll = nterms == 0 ? 0.0
                                : -0.5 * (nterms * LANE(s.per_term, v) + log(LANE(s.mant, v)) + s.expo[v] * M_LN2 +
                                          LANE(s.sumq, v));
        if (s.neg[v] || !isfinite(ll)) ll = -INFINITY;
        out[b0 + v] = ll;
    }
    free(Zc);
    free(Zfull);
}

/* ---------------- capacitance form, one candidate (TVλ, and ill-conditioned fixed Z) ---------------- */
static int capacitance_update(int M, int Mo, const params_t* p, const double* Z, const double* y, int N, double* beta,
                              double P[MMAX][MMAX], double* det_out, double* q_out) {
    double G[MMAX][MMAX] = {{0}}, u[MMAX] = {0}, vv = 0;
    for (int i = 0; i < N; ++i) {
        const double* Zi = Z + (size_t)i * M;
        double v = y[i];
        for (int l = 0; l < Mo; ++l) v -= Zi[l] * beta[l];
        vv += v * v;
        for (int a = 0; a < M; ++a) {
            u[a] += Zi[a] * v;
            for (int c = a; c < M; ++c) G[a][c] += Zi[a] * Zi[c];
        }
    }
    double A[MMAX * MMAX], W[MMAX * MMAX];
    for (int a = 0; a < M; ++a)
        for (int c = 0; c < M; ++c) {
            double s = a == c ? p->sig2 : 0.0;
            for (int l = 0; l < M; ++l) s += P[a][l] * (l <= c ? G[l][c] : G[c][l]);
            A[a * M + c] = s;
            W[a * M + c] = P[a][c];
        }
    double det = gauss(A, M, W, M);
    *det_out = det;
    if (det == 0.0) return 0;
    double uk = 0, bf[MMAX];
    for (int a = 0; a < M; ++a) {
        double s = 0;
        for (int c = 0; c < M; ++c) s += 0.5 * (W[a * M + c] + W[c * M + a]) * u[c];
        bf[a] = beta[a] + s;
        uk += u[a] * s;
    }
    *q_out = (vv - uk) / p->sig2;
    double T1[MMAX][MMAX];
    for (int a = 0; a < M; ++a) {
        double s = p->delta[a];
        for (int c = 0; c < M; ++c) s += p->Phi[a][c] * bf[c];
        beta[a] = s;
        for (int c = 0; c < M; ++c) {
            double x = 0;
            for (int l = 0; l < M; ++l) x += p->Phi[a][l] * 0.5 * (W[l * M + c] + W[c * M + l]);
            T1[a][c] = x;
        }
    }
    for (int a = 0; a < M; ++a)
        for (int c = a; c < M; ++c) {
            double x = 0;
            for (int l = 0; l < M; ++l) x += T1[a][l] * p->Phi[c][l];
            P[a][c] = P[c][a] = p->sig2 * x + p->Q[a][c];
        }
    return 1;
}

static void predict_one(int M, const params_t* p, double* beta, double P[MMAX][MMAX]) {
    double nb[MMAX], A[MMAX][MMAX];
    for (int i = 0; i < M; ++i) {
        double y = p->delta[i];
        for (int j = 0; j < M; ++j) y += p->Phi[i][j] * beta[j];
        nb[i] = y;
        for (int j = 0; j < M; ++j) {
            double z = 0;
            for (int l = 0; l < M; ++l) z += p->Phi[i][l] * P[l][j];
            A[i][j] = z;
        }
    }
    for (int i = 0; i < M; ++i) {
        beta[i] = nb[i];
        for (int j = i; j < M; ++j) {
            double z = p->Q[i][j];
            for (int l = 0; l < M; ++l) z += A[i][l] * p->Phi[j][l];
            P[i][j] = P[j][i] = z;
        }
    }
}

/* get_loss in the capacitance form for one candidate; Z (N×M row-major) fixed unless TVλ */
static double capacitance_run(int kind, const params_t* p, double* Z, const double* Y, int N, int nobs,
                              const double* mats) {
    const int M = state_dim(kind), Mo = kind == KIND_TVL ? 3 : M;
    double beta[MMAX], P[MMAX][MMAX];
    if (!init_state(M, p, beta, P)) return NAN;
    double ld = 0, sq = 0, last_ld = -INFINITY, last_q = 0;
    int neg = 0, last_neg = 0;
    for (int t = 0; t < nobs - 1; ++t) {
        const double* y = Y + (size_t)t * N;
        int nan = 0;
        for (int i = 0; i < N; ++i) nan |= isnan(y[i]);
        if (nan) {
            predict_one(M, p, beta, P);
        } else {
            if (kind == KIND_TVL) { /* tvλdns.jl:53-64, filter.jl:38-46 (dZ1 as written) */
                double lam = 1e-2 + exp(beta[3]), dl = lam - 1e-2, c1 = beta[1] + beta[2];
                for (int i = 0; i < N; ++i) {
                    double m = mats[i], tau = lam * m, z = exp(-tau), s = (1.0 - z) / tau;
                    double* Zi = Z + (size_t)i * M;
                    Zi[0] = 1.0;
                    Zi[1] = s;
                    Zi[2] = s - z;
                    Zi[3] = (c1 * (z / lam - z / (lam * lam * m)) + beta[2] * m * z) * dl;
                }
            }
            double det, q = NAN;
            int upd = capacitance_update(M, Mo, p, Z, y, N, beta, P, &det, &q);
            last_ld = upd ? (N - M) * log(p->sig2) + log(fabs(det)) : -INFINITY;
            last_q = upd ? q : NAN;
            last_neg = det < 0.0;
        }
        if (t >= 1) {
            ld += last_ld;
            sq += last_q;
            neg |= last_neg;
        }
    }
    const int nterms = nobs - 2 > 0 ? nobs - 2 : 0;
    double ll = nterms == 0 ? 0.0 : -0.5 * (ld + sq + nterms * N * log(2.0 * M_PI));
    if (neg || !isfinite(ll)) ll = -INFINITY;
    return ll;
}

static double capacitance_one(int kind, const params_t* p, const double* Z, const double* Y, int N, int nobs) {
    const int M = state_dim(kind);
    double* Zw = malloc(sizeof(double) * (size_t)N * M);
    memcpy(Zw, Z, sizeof(double) * (size_t)N * M);
    double ll = capacitance_run(kind, p, Zw, Y, N, nobs, NULL);
    free(Zw);
    return ll;
}

int yfm_cpu_fast_loglik(int kind, int space, const double* Y, int N, int T, const double* mats,
                        const double* theta, int P, int B, const int* T_use, double* out, int nthreads) {
    (void)P;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    if (kind == KIND_TVL) {
#pragma omp parallel
        {
            double* Z = malloc(sizeof(double) * (size_t)N * 4);
#pragma omp for schedule(dynamic, 1)
            for (int b = 0; b < B; ++b) {
                params_t p;
                decode(kind, theta + (size_t)b * param_count(kind), space, &p);
                out[b] = capacitance_run(kind, &p, Z, Y, N, T_use ? T_use[b] : T, mats);
            }
            free(Z);
        }
        return 0;
    }
    /* the centered panel columns (shared): ỹ = y − ȳ1, ȳ, ỹ'ỹ, NaN flags */
    double* Yc = malloc(sizeof(double) * (size_t)N * T);
    double* ybar = malloc(sizeof(double) * T);
    double* ytt = malloc(sizeof(double) * T);
    unsigned char* nanc = malloc(T);
    for (int t = 0; t < T; ++t) {
        const double* y = Y + (size_t)t * N;
        double s = 0;
        int nan = 0;
        for (int i = 0; i < N; ++i) { s += y[i]; nan |= isnan(y[i]); }
        ybar[t] = s / N;
        double q = 0;
        for (int i = 0; i < N; ++i) {
            double c = y[i] - ybar[t];
            Yc[(size_t)t * N + i] = c;
            q += c * c;
        }
        ytt[t] = q;
        nanc[t] = nan;
    }
    const int nblk = (B + V - 1) / V;
#pragma omp parallel for schedule(dynamic, 1)
    for (int k = 0; k < nblk; ++k) {
        const int b0 = k * V, nb = B - b0 < V ? B - b0 : V;
        fixedz_block(kind, Y, Yc, ybar, ytt, nanc, N, T, mats, theta, space, b0, nb, T_use, out);
    }
    free(Yc);
    free(ybar);
    free(ytt);
    free(nanc);
    return 0;
}

/*
 * yfm_oracle.c — reference-faithful CPU restatement of the YieldFactorModels.jl
 * Kalman log-likelihood (dense N×N path), in plain C with OpenMP over candidates.
 *
 * TEST INFRASTRUCTURE ONLY: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load this library, as the checker / the timed CPU baseline.
 * The product (libyfm_hip.so) never links or calls it.
 *
 * Parity status: parity unpinned against the Julia reference (no julia binary in
 * this image or on the GPU box, no reference fixtures).  It is
 * cross-checked against oracle/kalman_oracle.py (NumPy + LAPACK) and against
 * closed-form known answers in tests/test_oracle.py.
 *
 * What it restates (paths relative to the reference root):
 *   transform_params          src/models/parameteroperations.jl:22-32,
 *                             src/models/kalman/kalmanbasemodel.jl:74-120,
 *                             src/utils/transformations.jl:2-26
 *   set_params!               src/models/kalman/paramoperations.jl:6-68
 *   update_factor_loadings!   src/models/kalman/dns.jl:51-65, tvλdns.jl:53-64
 *   initialize_filter         src/models/kalman/filter.jl:1-10
 *   filter! (DNS)             src/models/kalman/filter.jl:125-179
 *   filter! (TVλ EKF)         src/models/kalman/filter.jl:12-80
 *   get_loss                  src/models/kalman/filter.jl:182-209
 * Every step forms F = (ZP)Z' + σ²I, inverts it with getrf + getri (unblocked,
 * partial pivoting, like LAPACK dgetf2/dgetri), and takes logdet(F) from a second
 * LU — the reference's O(N³)-per-step arithmetic, which is what the CPU baseline
 * must cost.  Julia's `\` and `inv` dispatch on triangular/diagonal matrices is
 * kept (LinearAlgebra generic.jl / dense.jl).
 *
 * Build: gcc -O3 -march=native -fopenmp -shared -fPIC yfm_oracle.c -o libyfm_oracle.so -lm
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

/* column-major element access */
#define AT(A, ld, i, j) (A)[(size_t)(j) * (ld) + (i)]

static int state_dim(int kind) { return kind == KIND_DNS ? 3 : kind == KIND_TVL ? 4 : 5; }
static int n_lead(int kind) { return kind == KIND_DNS ? 1 : kind == KIND_TVL ? 0 : 2; }

int yfm_oracle_param_count(int kind) {
    int M = state_dim(kind);
    return n_lead(kind) + 1 + M * (M + 1) / 2 + M + M * M;
}

/* ---------------- dense LAPACK-like kernels (column-major) ---------------- */

/* dgetf2: A = P L U, returns info (0 ok, k>0 first exact-zero pivot, 1-based). */
static int getrf(double* A, int n, int* ipiv) {
    int info = 0;
    for (int j = 0; j < n; ++j) {
        int p = j;
        double amax = fabs(AT(A, n, j, j));
        for (int i = j + 1; i < n; ++i) {
            double a = fabs(AT(A, n, i, j));
            if (a > amax) { amax = a; p = i; }
        }
        ipiv[j] = p;
        if (AT(A, n, p, j) != 0.0) {
            if (p != j)
                for (int k = 0; k < n; ++k) {
                    double t = AT(A, n, j, k); AT(A, n, j, k) = AT(A, n, p, k); AT(A, n, p, k) = t;
                }
            double r = 1.0 / AT(A, n, j, j);
            for (int i = j + 1; i < n; ++i) AT(A, n, i, j) *= r;
        } else if (info == 0) {
            info = j + 1;
        }
        for (int k = j + 1; k < n; ++k) {
            double akj = AT(A, n, j, k);
            if (akj != 0.0)
                for (int i = j + 1; i < n; ++i) AT(A, n, i, k) -= AT(A, n, i, j) * akj;
        }
    }
    return info;
}

/* dtrti2 (upper, non-unit): in-place inverse of the upper triangle. */
static int trtri_upper(double* A, int n) {
    for (int j = 0; j < n; ++j) if (AT(A, n, j, j) == 0.0) return j + 1;
    for (int j = 0; j < n; ++j) {
        AT(A, n, j, j) = 1.0 / AT(A, n, j, j);
        double ajj = -AT(A, n, j, j);
        /* x = A[0:j, j]; x := triu(A[0:j,0:j]) x  (dtrmv upper, no-trans) */
        for (int k = 0; k < j; ++k) {
            double temp = AT(A, n, k, j);
            if (temp != 0.0) {
                for (int i = 0; i < k; ++i) AT(A, n, i, j) += temp * AT(A, n, i, k);
                AT(A, n, k, j) = temp * AT(A, n, k, k);
            }
        }
        for (int i = 0; i < j; ++i) AT(A, n, i, j) *= ajj;
    }
    return 0;
}

/* dtrti2 (lower, non-unit). */
static int trtri_lower(double* A, int n) {
    for (int j = 0; j < n; ++j) if (AT(A, n, j, j) == 0.0) return j + 1;
    for (int j = n - 1; j >= 0; --j) {
        AT(A, n, j, j) = 1.0 / AT(A, n, j, j);
        double ajj = -AT(A, n, j, j);
        if (j < n - 1) {
            /* x = A[j+1:n, j]; x := tril(A[j+1:n, j+1:n]) x (dtrmv lower, no-trans) */
            for (int k = n - 1; k > j; --k) {
                double temp = AT(A, n, k, j);
                if (temp != 0.0) {
                    for (int i = n - 1; i > k; --i) AT(A, n, i, j) += temp * AT(A, n, i, k);
                    AT(A, n, k, j) = temp * AT(A, n, k, k);
                }
            }
            for (int i = j + 1; i < n; ++i) AT(A, n, i, j) *= ajj;
        }
    }
    return 0;
}

/* dgetri (unblocked): inverse from the LU factors; work has n doubles. */
static void getri(double* A, int n, const int* ipiv, double* work) {
    trtri_upper(A, n); /* U^{-1} (nonsingular: caller checked getrf info) */
    for (int j = n - 1; j >= 0; --j) {
        for (int i = j + 1; i < n; ++i) { work[i] = AT(A, n, i, j); AT(A, n, i, j) = 0.0; }
        if (j < n - 1) /* A[:, j] -= A[:, j+1:n] * work[j+1:n]  (dgemv) */
            for (int k = j + 1; k < n; ++k) {
                double w = work[k];
                for (int i = 0; i < n; ++i) AT(A, n, i, j) -= AT(A, n, i, k) * w;
            }
    }
    for (int j = n - 2; j >= 0; --j) {
        int jp = ipiv[j];
        if (jp != j)
            for (int i = 0; i < n; ++i) {
                double t = AT(A, n, i, j); AT(A, n, i, j) = AT(A, n, i, jp); AT(A, n, i, jp) = t;
            }
    }
}

static int is_triu(const double* A, int n) {
    for (int j = 0; j < n; ++j) for (int i = j + 1; i < n; ++i) if (AT(A, n, i, j) != 0.0) return 0;
    return 1;
}
static int is_tril(const double* A, int n) {
    for (int j = 0; j < n; ++j) for (int i = 0; i < j; ++i) if (AT(A, n, i, j) != 0.0) return 0;
    return 1;
}

/* Julia inv(A::StridedMatrix) (dense.jl): triangular inverse or getrf+getri. 0 ok, 1 singular. */
static int jl_inv(double* A, int n, int* ipiv, double* work) {
    if (is_triu(A, n)) return trtri_upper(A, n) ? 1 : 0;
    if (is_tril(A, n)) return trtri_lower(A, n) ? 1 : 0;
    if (getrf(A, n, ipiv)) return 1;
    getri(A, n, ipiv, work);
    return 0;
}

/* Julia A \ b (generic.jl): Diagonal / triangular / LU. A is destroyed. 0 ok, 1 singular. */
static int jl_ldiv(double* A, int n, double* b, int* ipiv) {
    int lo = is_tril(A, n), up = is_triu(A, n);
    if (lo && up) {
        for (int i = 0; i < n; ++i) if (AT(A, n, i, i) == 0.0) return 1;
        for (int i = 0; i < n; ++i) b[i] = b[i] / AT(A, n, i, i);
        return 0;
    }
    if (lo) {
        for (int i = 0; i < n; ++i) if (AT(A, n, i, i) == 0.0) return 1;
        for (int j = 0; j < n; ++j) {
            b[j] /= AT(A, n, j, j);
            for (int i = j + 1; i < n; ++i) b[i] -= b[j] * AT(A, n, i, j);
        }
        return 0;
    }
    if (up) {
        for (int i = 0; i < n; ++i) if (AT(A, n, i, i) == 0.0) return 1;
        for (int j = n - 1; j >= 0; --j) {
            b[j] /= AT(A, n, j, j);
            for (int i = 0; i < j; ++i) b[i] -= b[j] * AT(A, n, i, j);
        }
        return 0;
    }
    if (getrf(A, n, ipiv)) return 1;
    for (int i = 0; i < n; ++i) { int p = ipiv[i]; if (p != i) { double t = b[i]; b[i] = b[p]; b[p] = t; } }
    for (int j = 0; j < n; ++j) for (int i = j + 1; i < n; ++i) b[i] -= b[j] * AT(A, n, i, j);
    for (int j = n - 1; j >= 0; --j) {
        b[j] /= AT(A, n, j, j);
        for (int i = 0; i < j; ++i) b[i] -= b[j] * AT(A, n, i, j);
    }
    return 0;
}

/* Julia logdet(A): LU (check=false); singular -> -Inf; det<0 -> DomainError (returns 1). */
static int jl_logdet(double* A, int n, int* ipiv, double* out) {
    int info = getrf(A, n, ipiv);
    if (info) { *out = -INFINITY; return 0; }
    double s = 1.0, acc = 0.0;
    for (int i = 0; i < n; ++i) {
        double d = AT(A, n, i, i);
        s *= (d > 0) ? 1.0 : (d < 0) ? -1.0 : (d == 0 ? 0.0 : NAN);
        if (ipiv[i] != i) s = -s;
        acc += log(fabs(d));
    }
    if (s < 0) return 1;
    *out = acc + log(s);
    return 0;
}

/* ------------------------------- the model ------------------------------- */
typedef struct {
    int kind, N, M;
    const double* mats;
    double *Z, *ypred, *v, *F, *Finv, *Fw, *tNM, *tMN, *work, *zi;
    int* ipiv;
    double beta[MMAX], delta[MMAX], Phi[MMAX * MMAX], Q[MMAX * MMAX], P[MMAX * MMAX];
    double sigma2, lam;
} model_t;

static void model_alloc(model_t* m, int kind, int N, const double* mats) {
    m->kind = kind; m->N = N; m->M = state_dim(kind); m->mats = mats;
    size_t NN = (size_t)N * N;
    m->Z = calloc((size_t)N * MMAX, sizeof(double));
    m->ypred = calloc(N, sizeof(double));
    m->v = calloc(N, sizeof(double));
    m->F = calloc(NN, sizeof(double));
    m->Finv = calloc(NN, sizeof(double));
    m->Fw = calloc(NN, sizeof(double));
    m->tNM = calloc((size_t)N * MMAX, sizeof(double));
    m->tMN = calloc((size_t)N * MMAX, sizeof(double));
    m->work = calloc(N > 32 ? N : 32, sizeof(double));
    m->zi = calloc(N, sizeof(double));
    m->ipiv = calloc(N > 32 ? N : 32, sizeof(int));
}
static void model_free(model_t* m) {
    free(m->Z); free(m->ypred); free(m->v); free(m->F); free(m->Finv); free(m->Fw);
    free(m->tNM); free(m->tMN); free(m->work); free(m->zi); free(m->ipiv);
}
static void model_reset(model_t* m) {
    int N = m->N, M = m->M;
    for (int i = 0; i < N * M; ++i) m->Z[i] = 1.0; /* kalmanbasemodel.jl:53 */
    memset(m->F, 0, sizeof(double) * N * N);
    memset(m->Finv, 0, sizeof(double) * N * N);
    memset(m->v, 0, sizeof(double) * N);
}

static double from_R_to_11(double x) { double y = exp(x); return 2.0 * y / (1.0 + y) - 1.0; }

static void loadings_pair(const double* mats, int N, double g, double* Zs, double* Zc) {
    double lam = 1e-2 + exp(g); /* dns.jl:51-65 */
    for (int i = 0; i < N; ++i) {
        double tau = lam * mats[i];
        double z = exp(-tau);
        Zs[i] = (1.0 - z) / tau;
        Zc[i] = Zs[i] - z;
    }
}

/* transform_params + set_params! ; theta has P entries */
static void set_params(model_t* m, const double* theta, int space) {
    int M = m->M, N = m->N, L = n_lead(m->kind);
    double tc[64];
    int P = yfm_oracle_param_count(m->kind);
    for (int i = 0; i < P; ++i) tc[i] = theta[i];
    if (space == 0) { /* kalmanbasemodel.jl:106-112 */
        int k = L;
        tc[k] = exp(tc[k]); k++;
        for (int j = 0; j < M; ++j) for (int i = 0; i <= j; ++i, ++k) if (i == j) tc[k] = exp(tc[k]);
        k += M;
        for (int i = 0; i < M; ++i) for (int j = 0; j < M; ++j, ++k) if (i == j) tc[k] = from_R_to_11(tc[k]);
    }
    int k = L;
    m->sigma2 = tc[k++];
    double U[MMAX * MMAX] = {0};
    for (int j = 0; j < M; ++j) for (int i = 0; i <= j; ++i) U[j * M + i] = tc[k++];
    for (int j = 0; j < M; ++j) for (int i = 0; i < M; ++i) { /* Q = U'U */
        double s = 0; for (int l = 0; l < M; ++l) s += U[i * M + l] * U[j * M + l];
        m->Q[j * M + i] = s;
    }
    for (int i = 0; i < M; ++i) m->delta[i] = tc[k++];
    for (int i = 0; i < M; ++i) for (int j = 0; j < M; ++j) m->Phi[j * M + i] = tc[k++]; /* row-major */
    if (m->kind == KIND_DNS) {
        for (int i = 0; i < N; ++i) m->Z[i] = 1.0;
        loadings_pair(m->mats, N, tc[0], m->Z + N, m->Z + 2 * N);
    } else if (m->kind == KIND_GNS) {
        for (int i = 0; i < N; ++i) m->Z[i] = 1.0;
        loadings_pair(m->mats, N, tc[0], m->Z + N, m->Z + 2 * N);
        loadings_pair(m->mats, N, tc[1], m->Z + 3 * N, m->Z + 4 * N);
    }
}

/* filter.jl:1-10 ; returns 1 if it would throw */
static int initialize_filter(model_t* m) {
    int M = m->M, M2 = M * M;
    double A[MMAX * MMAX], b[MMAX];
    for (int j = 0; j < M; ++j) for (int i = 0; i < M; ++i) A[j * M + i] = (i == j) - m->Phi[j * M + i];
    for (int i = 0; i < M; ++i) b[i] = m->delta[i];
    int ipiv[MMAX * MMAX];
    if (jl_ldiv(A, M, b, ipiv)) return 1;
    for (int i = 0; i < M; ++i) m->beta[i] = b[i];
    double K[MMAX * MMAX * MMAX * MMAX], work[MMAX * MMAX];
    /* I - kron(Phi, Phi), column-major M²×M² */
    for (int j1 = 0; j1 < M; ++j1) for (int j2 = 0; j2 < M; ++j2)
        for (int i1 = 0; i1 < M; ++i1) for (int i2 = 0; i2 < M; ++i2) {
            int r = i1 * M + i2, c = j1 * M + j2;
            K[c * M2 + r] = (r == c) - m->Phi[j1 * M + i1] * m->Phi[j2 * M + i2];
        }
    if (jl_inv(K, M2, ipiv, work)) return 1;
    for (int r = 0; r < M2; ++r) {
        double s = 0; for (int c = 0; c < M2; ++c) s += K[c * M2 + r] * m->Q[c];
        m->P[r] = s; /* vec -> reshape column-major */
    }
    return 0;
}

static void mm(const double* A, const double* B, double* C, int n, int k, int p) { /* C(n×p)=A(n×k)B(k×p) */
    for (int j = 0; j < p; ++j) for (int i = 0; i < n; ++i) {
        double s = 0; for (int l = 0; l < k; ++l) s += A[l * n + i] * B[j * k + l];
        C[j * n + i] = s;
    }
}

static void predict_only(model_t* m) {
    int M = m->M, N = m->N;
    double tb[MMAX], tP[MMAX * MMAX];
    for (int i = 0; i < N; ++i) { double s = 0; for (int l = 0; l < (m->kind == KIND_TVL ? 3 : M); ++l) s += m->Z[l * N + i] * m->beta[l]; m->ypred[i] = s; }
    for (int i = 0; i < M; ++i) { double s = 0; for (int l = 0; l < M; ++l) s += m->Phi[l * M + i] * m->beta[l]; tb[i] = s; }
    for (int i = 0; i < M; ++i) m->beta[i] = m->delta[i] + tb[i];
    mm(m->Phi, m->P, tP, M, M, M);
    for (int j = 0; j < M; ++j) for (int i = 0; i < M; ++i) {
        double s = 0; for (int l = 0; l < M; ++l) s += tP[l * M + i] * m->Phi[l * M + j];
        m->P[j * M + i] = s + m->Q[j * M + i];
    }
}

static void tvl_loadings(model_t* m, double b4) { /* tvλdns.jl:53-64 */
    int N = m->N;
    m->lam = 1e-2 + exp(b4);
    for (int i = 0; i < N; ++i) {
        double tau = m->lam * m->mats[i];
        m->zi[i] = exp(-tau);
        m->Z[N + i] = (1.0 - m->zi[i]) / tau;
        m->Z[2 * N + i] = m->Z[N + i] - m->zi[i];
    }
}

/* filter.jl:125-179 / :12-80. returns 0 normally, 1 if inv(F) threw */
static int filter_step(model_t* m, const double* y) {
    int N = m->N, M = m->M;
    int nan = 0;
    for (int i = 0; i < N; ++i) if (isnan(y[i])) nan = 1;
    if (m->kind == KIND_TVL) tvl_loadings(m, m->beta[3]);
    if (nan) { predict_only(m); return 0; }
    int Mo = m->kind == KIND_TVL ? 3 : M;
    for (int i = 0; i < N; ++i) {
        double s = 0; for (int l = 0; l < Mo; ++l) s += m->Z[l * N + i] * m->beta[l];
        m->ypred[i] = s; m->v[i] = y[i] - s;
    }
    if (m->kind == KIND_TVL) { /* filter.jl:38-46 (dZ1 quirk kept) */
        double dl = m->lam - 1e-2, lam = m->lam;
        for (int i = 0; i < N; ++i) {
            double z = m->zi[i], mt = m->mats[i];
            double dZ1 = z / lam - z / (lam * lam * mt);
            double dZ2 = mt * z;
            m->Z[3 * N + i] = ((m->beta[1] + m->beta[2]) * dZ1 + m->beta[2] * dZ2) * dl;
        }
    }
    mm(m->Z, m->P, m->tNM, N, M, M); /* ZP */
    for (int j = 0; j < N; ++j) for (int i = 0; i < N; ++i) { /* F = (ZP)Z' + σ²I */
        double s = 0; for (int l = 0; l < M; ++l) s += m->tNM[l * N + i] * m->Z[l * N + j];
        m->F[j * N + i] = s + (i == j ? m->sigma2 : 0.0);
    }
    memcpy(m->Fw, m->F, sizeof(double) * N * N);
    if (jl_inv(m->Fw, N, m->ipiv, m->work)) {
        if (m->kind != KIND_TVL) for (int i = 0; i < N * N; ++i) m->Finv[i] = INFINITY;
        return 1;
    }
    memcpy(m->Finv, m->Fw, sizeof(double) * N * N);
    /* K = (Z P')' F^{-1}  (M×N) */
    double Pt[MMAX * MMAX];
    for (int j = 0; j < M; ++j) for (int i = 0; i < M; ++i) Pt[j * M + i] = m->P[i * M + j];
    mm(m->Z, Pt, m->tNM, N, M, M);
    for (int j = 0; j < N; ++j) for (int i = 0; i < M; ++i) {
        double s = 0; for (int l = 0; l < N; ++l) s += m->tNM[i * N + l] * m->Finv[j * N + l];
        m->tMN[j * M + i] = s;
    }
    double tb[MMAX];
    for (int i = 0; i < M; ++i) { double s = 0; for (int l = 0; l < N; ++l) s += m->tMN[l * M + i] * m->v[l]; tb[i] = s; }
    for (int i = 0; i < M; ++i) m->beta[i] += tb[i];
    for (int i = 0; i < M; ++i) { double s = 0; for (int l = 0; l < M; ++l) s += m->Phi[l * M + i] * m->beta[l]; tb[i] = s; }
    for (int i = 0; i < M; ++i) m->beta[i] = m->delta[i] + tb[i];
    double KZ[MMAX * MMAX], IKZ[MMAX * MMAX], T1[MMAX * MMAX], T2[MMAX * MMAX];
    mm(m->tMN, m->Z, KZ, M, N, M);
    for (int i = 0; i < M * M; ++i) IKZ[i] = ((i % M) == (i / M)) - KZ[i];
    mm(IKZ, m->P, T1, M, M, M);
    mm(m->Phi, T1, T2, M, M, M);
    for (int j = 0; j < M; ++j) for (int i = 0; i < M; ++i) {
        double s = 0; for (int l = 0; l < M; ++l) s += T2[l * M + i] * m->Phi[l * M + j];
        m->P[j * M + i] = s + m->Q[j * M + i];
    }
    return 0;
}

/* filter.jl:182-209. returns loglik; NaN if initialize_filter would throw. */
static double get_loss(model_t* m, const double* Y, int ldy, int nobs, double* rec_beta, double* rec_P) {
    if (initialize_filter(m)) return NAN;
    int N = m->N, M = m->M;
    double ll = 0.0, logdet_2pi = N * log(2.0 * M_PI);
    for (int t = 1; t <= nobs - 1; ++t) {
        filter_step(m, Y + (size_t)(t - 1) * ldy);
        if (rec_beta) {
            memcpy(rec_beta + (size_t)(t - 1) * M, m->beta, sizeof(double) * M);
            memcpy(rec_P + (size_t)(t - 1) * M * M, m->P, sizeof(double) * M * M);
        }
        if (t > 1) {
            double ld;
            memcpy(m->Fw, m->F, sizeof(double) * N * N);
            if (jl_logdet(m->Fw, N, m->ipiv, &ld)) return -INFINITY;
            double q = 0;
            for (int j = 0; j < N; ++j) {
                double s = 0; for (int i = 0; i < N; ++i) s += m->v[i] * m->Finv[j * N + i];
                q += s * m->v[j];
            }
            ll -= 0.5 * (ld + q + logdet_2pi);
        }
        if (isinf(ll) || isnan(ll)) return -INFINITY;
    }
    return ll;
}

/*
 * Batched faithful loglik.  Y: N×T column-major; theta: P×B column-major;
 * T_use: B entries or NULL (columns 1..T_use[b] are used); out: B logliks.
 * nthreads <= 0 uses the OpenMP default.  Returns 0.
 */
int yfm_oracle_loglik(int kind, int space, const double* Y, int N, int T, const double* mats,
                      const double* theta, int P, int B, const int* T_use, double* out, int nthreads) {
    (void)P;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel
    {
        model_t m;
        model_alloc(&m, kind, N, mats);
        int Pk = yfm_oracle_param_count(kind);
#pragma omp for schedule(dynamic, 1)
        for (int b = 0; b < B; ++b) {
            int nobs = T_use ? T_use[b] : T;
            model_reset(&m);
            set_params(&m, theta + (size_t)b * Pk, space);
            out[b] = get_loss(&m, Y, N, nobs, NULL, NULL);
        }
        model_free(&m);
    }
    return 0;
}

/* One candidate with trajectories: beta_out (M×(T-1)), P_out (M×M×(T-1)), column-major. */
int yfm_oracle_filter_states(int kind, int space, const double* Y, int N, int T, const double* mats,
                             const double* theta, double* beta_out, double* P_out, double* loglik) {
    model_t m;
    model_alloc(&m, kind, N, mats);
    model_reset(&m);
    set_params(&m, theta, space);
    *loglik = get_loss(&m, Y, N, T, beta_out, P_out);
    model_free(&m);
    return 0;
}

/*
 * yfm_truth.c — quad-precision (binary128, 113-bit significand) ground truth of the
 * reference Kalman log-likelihood, for ADJUDICATING parity.
 *
 * TEST INFRASTRUCTURE ONLY: only tests/ and bench.py's cpu_baseline/parity leg load this
 * library, as a checker.  The product (libyfm_hip.so) never links or calls it.
 *
 * What "truth" means here: the reference's recursion evaluated in (nearly) exact
 * arithmetic on the same FP64 inputs (θ, panel, maturities, the FP64 literals 0.01 of
 * tvλdns.jl:56 / dns.jl:57).  It separates an FP64 implementation's own rounding from
 * a difference in what is computed: where the reference's dense FP64 path and the HIP
 * kernel disagree, the one closer to this value is the one closer to the reference
 * algorithm in exact arithmetic.  For the TVλ EKF that matters: some
 * candidates amplify an FP64 rounding by 1e10..1e13 over T = 600 steps, so two FP64
 * implementations of filter.jl:12-80 differ by up to 1e-4 relative — while a 113-bit
 * run is still ~1e-20 from exact.
 *
 * Algebra (exact identities): with G = Z'Z, u = Z'v,
 * B̃ = σ²I + P G, W = B̃⁻¹P:
 *   K v = W u,  (I − KZ)P = σ² W,  v'F⁻¹v = (v'v − u'Wu)/σ²,
 *   det F = σ^{2(N−M)} det B̃   (so sign det F = sign det B̃, and F is singular iff
 *   det B̃ = 0 or σ² = 0 with N > M).
 * This avoids the N×N inverse, so a 360-maturity candidate takes ~1 s instead of hours.
 * tests/test_oracle.py pins it to the 40-digit dense mpmath restatement
 * (oracle/kalman_mp.py, which forms F and inverts it as filter.jl does).
 *
 * Restates (paths relative to the reference root):
 *   transform_params / set_params!   src/models/parameteroperations.jl:22-32,
 *                                    src/models/kalman/paramoperations.jl:6-68,
 *                                    src/models/kalman/kalmanbasemodel.jl:74-120,
 *                                    src/utils/transformations.jl:2-26
 *   loadings                         src/models/kalman/dns.jl:51-65, tvλdns.jl:53-64
 *   initialize_filter                src/models/kalman/filter.jl:1-10 (M²×M² system)
 *   filter! DNS / TVλ                src/models/kalman/filter.jl:125-179 / :12-80
 *                                    (dZ1 = z/λ − z/(λ²m) kept as written, :43)
 *   get_loss                         src/models/kalman/filter.jl:182-209
 *
 * Build: gcc -O2 -fopenmp -shared -fPIC yfm_truth.c -o libyfm_truth.so -lquadmath -lm
 */
#include <math.h>
#include <quadmath.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef __float128 qd;

#define KIND_DNS 0
#define KIND_TVL 1
#define KIND_GNS 2
#define MMAX 5

static int state_dim(int kind) { return kind == KIND_DNS ? 3 : kind == KIND_TVL ? 4 : 5; }
static int n_lead(int kind) { return kind == KIND_DNS ? 1 : kind == KIND_TVL ? 0 : 2; }

int yfm_truth_param_count(int kind) {
    int M = state_dim(kind);
    return n_lead(kind) + 1 + M * (M + 1) / 2 + M + M * M;
}

/* Gaussian elimination with partial pivoting on an n×n row-major system with r
 * right-hand sides (row-major n×r).  Returns the determinant (0 on an exact zero pivot,
 * where LAPACK getrf reports info > 0). */
static qd gauss(qd* A, int n, qd* X, int r) {
    qd det = 1;
    for (int k = 0; k < n; ++k) {
        int p = k;
        qd amax = fabsq(A[k * n + k]);
        for (int i = k + 1; i < n; ++i)
            if (fabsq(A[i * n + k]) > amax) { amax = fabsq(A[i * n + k]); p = i; }
        if (A[p * n + k] == 0) return 0;
        if (p != k) {
            det = -det;
            for (int c = 0; c < n; ++c) { qd t = A[k * n + c]; A[k * n + c] = A[p * n + c]; A[p * n + c] = t; }
            for (int c = 0; c < r; ++c) { qd t = X[k * r + c]; X[k * r + c] = X[p * r + c]; X[p * r + c] = t; }
        }
        det *= A[k * n + k];
        for (int i = k + 1; i < n; ++i) {
            qd l = A[i * n + k] / A[k * n + k];
            for (int c = k + 1; c < n; ++c) A[i * n + c] -= l * A[k * n + c];
            for (int c = 0; c < r; ++c) X[i * r + c] -= l * X[k * r + c];
        }
    }
    for (int k = n - 1; k >= 0; --k)
        for (int c = 0; c < r; ++c) {
            qd s = X[k * r + c];
            for (int j = k + 1; j < n; ++j) s -= A[k * n + j] * X[j * r + c];
            X[k * r + c] = s / A[k * n + k];
        }
    return det;
}

typedef struct {
    int kind, N, M, lead;
    qd sig2, gam[2], Q[MMAX][MMAX], delta[MMAX], Phi[MMAX][MMAX];
    qd beta[MMAX], P[MMAX][MMAX];
    qd *mats, *Z; /* Z: N×MMAX row-major (row i = maturity i) */
} tmodel;

static void decode(tmodel* m, const double* th, int space) {
    int M = m->M, k = 0;
    for (int l = 0; l < m->lead; ++l) m->gam[l] = th[k++];
    m->sig2 = space == 0 ? expq((qd)th[k]) : (qd)th[k];
    ++k;
    qd U[MMAX][MMAX];
    memset(U, 0, sizeof U);
    for (int j = 0; j < M; ++j)
        for (int i = 0; i <= j; ++i) {
            qd x = th[k++];
            U[i][j] = (i == j && space == 0) ? expq(x) : x;
        }
    for (int i = 0; i < M; ++i)
        for (int j = 0; j < M; ++j) {
            qd s = 0;
            for (int l = 0; l < M; ++l) s += U[l][i] * U[l][j]; /* Q = U'U */
            m->Q[i][j] = s;
        }
    for (int i = 0; i < M; ++i) m->delta[i] = th[k++];
    for (int i = 0; i < M; ++i)
        for (int j = 0; j < M; ++j) {
            qd x = th[k++];
            if (i == j && space == 0) { qd y = expq(x); x = 2 * y / (1 + y) - 1; } /* from_R_to_11 */
            m->Phi[i][j] = x; /* row-major reshape' */
        }
}

/* Z[:, 1+2l], Z[:, 2+2l] for a fixed λ = 0.01 + e^γ (dns.jl:51-65) */
static void loadings_pair(tmodel* m, qd lam, int col) {
    for (int i = 0; i < m->N; ++i) {
        qd tau = lam * m->mats[i], z = expq(-tau);
        qd s = (1 - z) / tau;
        m->Z[i * MMAX + col] = s;
        m->Z[i * MMAX + col + 1] = s - z;
    }
}

/* filter.jl:1-10 ; returns 0 where the reference would throw */
static int init_filter(tmodel* m) {
    int M = m->M, M2 = M * M;
    qd A[MMAX * MMAX], b[MMAX];
    for (int i = 0; i < M; ++i) {
        for (int j = 0; j < M; ++j) A[i * M + j] = (i == j) - m->Phi[i][j];
        b[i] = m->delta[i];
    }
    if (gauss(A, M, b, 1) == 0) return 0;
    for (int i = 0; i < M; ++i) m->beta[i] = b[i];
    qd K[MMAX * MMAX * MMAX * MMAX], vq[MMAX * MMAX];
    for (int i1 = 0; i1 < M; ++i1) /* (I − Φ⊗Φ) vec P = vec Q, vec column-major */
        for (int i2 = 0; i2 < M; ++i2)
            for (int j1 = 0; j1 < M; ++j1)
                for (int j2 = 0; j2 < M; ++j2) {
                    int r = i1 * M + i2, c = j1 * M + j2;
                    K[r * M2 + c] = (r == c) - m->Phi[i1][j1] * m->Phi[i2][j2];
                }
    for (int r = 0; r < M2; ++r) vq[r] = m->Q[r % M][r / M];
    if (gauss(K, M2, vq, 1) == 0) return 0;
    for (int r = 0; r < M2; ++r) m->P[r % M][r / M] = vq[r];
    return 1;
}

static void predict_only(tmodel* m) {
    int M = m->M;
    qd b[MMAX], A[MMAX][MMAX];
    for (int i = 0; i < M; ++i) {
        qd s = m->delta[i];
        for (int j = 0; j < M; ++j) s += m->Phi[i][j] * m->beta[j];
        b[i] = s;
        for (int j = 0; j < M; ++j) {
            qd a = 0;
            for (int l = 0; l < M; ++l) a += m->Phi[i][l] * m->P[l][j];
            A[i][j] = a;
        }
    }
    for (int i = 0; i < M; ++i) {
        m->beta[i] = b[i];
        for (int j = 0; j < M; ++j) {
            qd s = m->Q[i][j];
            for (int l = 0; l < M; ++l) s += A[i][l] * m->Phi[j][l];
            m->P[i][j] = s;
        }
    }
}

/* One update step on column y (no NaN).  Returns 0 if F is singular in exact arithmetic
 * (the reference's inv(F) throws: no update), else 1; *logdetF / *signF / *q get the
 * get_loss terms of the new F and v. */
static int update(tmodel* m, const double* y, qd* logabsdet, int* sign, qd* q) {
    int N = m->N, M = m->M;
    const int Mo = m->kind == KIND_TVL ? 3 : M; /* ŷ = Z[:,1:3]β[1:3] for TVλ (filter.jl:33) */
    if (m->kind == KIND_TVL) {
        qd e4 = expq(m->beta[3]);
        qd lam = (qd)1e-2 + e4; /* tvλdns.jl:56 */
        qd dl = lam - (qd)1e-2; /* filter.jl:38 */
        qd c1 = m->beta[1] + m->beta[2];
        for (int i = 0; i < N; ++i) {
            qd mt = m->mats[i], tau = lam * mt, z = expq(-tau);
            qd s = (1 - z) / tau;
            qd *Zi = m->Z + i * MMAX;
            Zi[0] = 1;
            Zi[1] = s;
            Zi[2] = s - z;
            qd dz1 = z / lam - z / (lam * lam * mt); /* filter.jl:43, as written */
            qd dz2 = mt * z;                         /* :44 */
            Zi[3] = (c1 * dz1 + m->beta[2] * dz2) * dl; /* :46 */
        }
    }
    qd G[MMAX][MMAX], u[MMAX], vv = 0;
    memset(G, 0, sizeof G);
    memset(u, 0, sizeof u);
    for (int i = 0; i < N; ++i) {
        const qd* Zi = m->Z + i * MMAX;
        qd v = y[i];
        for (int l = 0; l < Mo; ++l) v -= Zi[l] * m->beta[l];
        vv += v * v;
        for (int a = 0; a < M; ++a) {
            u[a] += Zi[a] * v;
            for (int c = 0; c < M; ++c) G[a][c] += Zi[a] * Zi[c];
        }
    }
    qd A[MMAX * MMAX], W[MMAX * MMAX];
    for (int i = 0; i < M; ++i)
        for (int j = 0; j < M; ++j) {
            qd s = (i == j) ? m->sig2 : 0;
            for (int l = 0; l < M; ++l) s += m->P[i][l] * G[l][j];
            A[i * M + j] = s;
            W[i * M + j] = m->P[i][j];
        }
    qd det = gauss(A, M, W, M);
    if (det == 0 || (m->sig2 == 0 && N > M)) {
        *logabsdet = -INFINITY;
        *sign = 1;
        *q = 0;
        return 0;
    }
    *sign = det < 0 ? -1 : 1;
    *logabsdet = (N - M) * logq(m->sig2) + logq(fabsq(det));
    qd kv[MMAX], uk = 0;
    for (int i = 0; i < M; ++i) {
        qd s = 0;
        for (int j = 0; j < M; ++j) s += W[i * M + j] * u[j];
        kv[i] = s;
        uk += u[i] * s;
    }
    *q = (vv - uk) / m->sig2;
    qd bf[MMAX];
    for (int i = 0; i < M; ++i) bf[i] = m->beta[i] + kv[i];
    qd T1[MMAX][MMAX];
    for (int i = 0; i < M; ++i) {
        qd s = m->delta[i];
        for (int j = 0; j < M; ++j) s += m->Phi[i][j] * bf[j];
        m->beta[i] = s;
        for (int j = 0; j < M; ++j) {
            qd a = 0;
            for (int l = 0; l < M; ++l) a += m->Phi[i][l] * W[l * M + j];
            T1[i][j] = a;
        }
    }
    for (int i = 0; i < M; ++i)
        for (int j = 0; j < M; ++j) {
            qd s = 0;
            for (int l = 0; l < M; ++l) s += T1[i][l] * m->Phi[j][l];
            m->P[i][j] = m->sig2 * s + m->Q[i][j]; /* Φ(I−KZ)PΦ' + Q, (I−KZ)P = σ²W */
        }
    return 1;
}

/* get_loss (filter.jl:182-209) for one candidate on Y[:, 1:nobs]; NaN where the reference
 * throws from initialize_filter.  rec_beta / rec_P (or NULL): state after every filter! call
 * (M×(nobs−1) and M×M×(nobs−1), column-major). */
static double get_loss(tmodel* m, const double* Y, int ldy, int nobs, double* rec_beta, double* rec_P) {
    int N = m->N, M = m->M;
    if (!init_filter(m)) return NAN;
    const qd c2pi = (qd)N * logq(2 * M_PIq);
    qd ll = 0, last_ld = -INFINITY, last_q = 0; /* fresh model: F = 0, F⁻¹ = 0, v = 0 */
    int last_sign = 1, dead = 0;
    for (int t = 1; t <= nobs - 1; ++t) {
        const double* y = Y + (size_t)(t - 1) * ldy;
        int nan = 0;
        for (int i = 0; i < N; ++i) nan |= isnan(y[i]);
        if (nan) {
            predict_only(m); /* F, F⁻¹, v stale (filter.jl:13-29, :126-140) */
        } else {
            qd lad, q;
            int sg;
            update(m, y, &lad, &sg, &q);
            last_ld = lad;
            last_sign = sg;
            last_q = q;
        }
        if (rec_beta) {
            for (int i = 0; i < M; ++i) {
                rec_beta[(size_t)(t - 1) * M + i] = (double)m->beta[i];
                for (int j = 0; j < M; ++j) rec_P[(size_t)(t - 1) * M * M + j * M + i] = (double)m->P[i][j];
            }
        }
        if (t > 1 && !dead) {
            if (last_sign < 0) dead = 1; /* logdet DomainError */
            else {
                ll -= (last_ld + last_q + c2pi) / 2;
                if (isinfq(ll) || isnanq(ll)) dead = 1;
            }
        }
    }
    return dead ? -INFINITY : (double)ll;
}

static void model_init(tmodel* m, int kind, int N, const double* mats) {
    m->kind = kind;
    m->N = N;
    m->M = state_dim(kind);
    m->lead = n_lead(kind);
    m->mats = malloc(sizeof(qd) * (size_t)N);
    m->Z = malloc(sizeof(qd) * (size_t)N * MMAX);
    for (int i = 0; i < N; ++i) m->mats[i] = mats[i];
}

static void model_set(tmodel* m, const double* theta, int space) {
    decode(m, theta, space);
    for (int i = 0; i < m->N; ++i) m->Z[i * MMAX] = 1;
    for (int l = 0; l < m->lead; ++l) loadings_pair(m, (qd)1e-2 + expq(m->gam[l]), 1 + 2 * l);
}

/* Batched truth loglik: Y N×T column-major, theta P×B column-major, T_use (B) or NULL. */
int yfm_truth_loglik(int kind, int space, const double* Y, int N, int T, const double* mats, const double* theta,
                     int P, int B, const int* T_use, double* out, int nthreads) {
    (void)P;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel
    {
        tmodel m;
        model_init(&m, kind, N, mats);
        const int Pk = yfm_truth_param_count(kind);
#pragma omp for schedule(dynamic, 1)
        for (int b = 0; b < B; ++b) {
            model_set(&m, theta + (size_t)b * Pk, space);
            out[b] = get_loss(&m, Y, N, T_use ? T_use[b] : T, NULL, NULL);
        }
        free(m.mats);
        free(m.Z);
    }
    return 0;
}

/* One candidate with its state trajectory (the layout of yfm_oracle_filter_states). */
int yfm_truth_filter_states(int kind, int space, const double* Y, int N, int T, const double* mats,
                            const double* theta, double* beta_out, double* P_out, double* loglik) {
    tmodel m;
    model_init(&m, kind, N, mats);
    model_set(&m, theta, space);
    *loglik = get_loss(&m, Y, N, T, beta_out, P_out);
    free(m.mats);
    free(m.Z);
    return 0;
}

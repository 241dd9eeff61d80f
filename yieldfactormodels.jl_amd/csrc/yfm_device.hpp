// yfm_device.hpp — device-side building blocks for the batched Kalman log-likelihood.
//
// Everything here is per-lane FP64 scalar code on fixed-size (compile-time M)
// arrays: the compiler fully unrolls it and keeps the state in VGPRs.  Row/column
// pivot choices are runtime values, realised as selects (no scratch indexing).
//
// Reference semantics restated (paths relative to the reference root):
//   decode_params    src/models/parameteroperations.jl:22-32 (transform_params),
//                    src/models/kalman/kalmanbasemodel.jl:74-120 (transform order),
//                    src/models/kalman/paramoperations.jl:6-59 (set_params!),
//                    src/utils/transformations.jl:2-26
//   init_state       src/models/kalman/filter.jl:1-10 (initialize_filter)
//   capacitance_*    the F = ZPZ' + σ²I solve of filter.jl:147-176 in capacitance
//                    (Woodbury) form: see DESIGN.md §3 for the algebra.
#pragma once
#include <hip/hip_runtime.h>

#include "yfm_flags.hpp"

namespace yfm {

constexpr double kLog2Pi = 1.8378770664093454835606594728112;  // log(2π)
constexpr double kLn2 = 0.69314718055994530941723212145818;

__device__ __forceinline__ double from_R_to_11(double x) {
  // transformations.jl:21-26, evaluated exactly as written (x > ~709.78 gives Inf/Inf = NaN)
  const double y = exp(x);
  return 2.0 * y / (1.0 + y) - 1.0;
}

template <int M, int LEAD>
struct Params {
  double gam[LEAD > 0 ? LEAD : 1];
  double sigma2;
  double Q[M][M];
  double delta[M];
  double Phi[M][M];
};

constexpr int param_count(int M, int lead) { return lead + 1 + M * (M + 1) / 2 + M + M * M; }

// transform_params (space == 0) + set_params!: θ layout [γ…, σ², U by column (i ≤ j), δ, Φ row-major].
template <int M, int LEAD>
__device__ __forceinline__ void decode_params(const double* __restrict__ th, int space, Params<M, LEAD>& p) {
  int k = 0;
#pragma unroll
  for (int l = 0; l < LEAD; ++l) p.gam[l] = th[k++];
  // (the exps are computed unconditionally and selected: a branch on `space` put each in its own block)
  const double e_s = exp(th[k]);
  p.sigma2 = space == 0 ? e_s : th[k];
  ++k;
  double U[M][M];
#pragma unroll
  for (int j = 0; j < M; ++j) {
#pragma unroll
    for (int i = 0; i < M; ++i) {
      if (i <= j) {
        double x = th[k++];
        if (i == j) {
          const double e = exp(x);
          x = space == 0 ? e : x;
        }
        U[i][j] = x;
      } else {
        U[i][j] = 0.0;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < M; ++i)
#pragma unroll
    for (int j = 0; j < M; ++j) {
      double s = 0.0;
#pragma unroll
      for (int l = 0; l < M; ++l) s = fma(U[l][i], U[l][j], s);  // Q = U'U (paramoperations.jl:35)
      p.Q[i][j] = s;
    }
#pragma unroll
  for (int i = 0; i < M; ++i) p.delta[i] = th[k++];
#pragma unroll
  for (int i = 0; i < M; ++i)
#pragma unroll
    for (int j = 0; j < M; ++j) {
      double x = th[k++];
      if (i == j) {
        const double e = from_R_to_11(x);
        x = space == 0 ? e : x;
      }
      p.Phi[i][j] = x;  // reshape(·, M, M)' == row-major (paramoperations.jl:38)
    }
}

// In-register Gaussian elimination with partial pivoting (LAPACK getf2 pivot rule:
// first index of max |a|), n×n with R right-hand sides.  Returns false on an exact
// zero pivot — where LAPACK's getrf reports info > 0 and Julia throws.
template <int n, int R>
__device__ __forceinline__ bool gauss_solve(double (&A)[n][n], double (&X)[n][R]) {
  bool ok = true;
#pragma unroll
  for (int k = 0; k < n; ++k) {
    // pivot search
    int p = k;
    double amax = fabs(A[k][k]);
#pragma unroll
    for (int i = k + 1; i < n; ++i) {
      const double a = fabs(A[i][k]);
      const bool gt = a > amax;
      amax = gt ? a : amax;
      p = gt ? i : p;
    }
    // swap rows k and p (selects)
#pragma unroll
    for (int i = k + 1; i < n; ++i) {
      const bool s = (p == i);
#pragma unroll
      for (int c = k; c < n; ++c) {
        const double a = A[k][c], b = A[i][c];
        A[k][c] = s ? b : a;
        A[i][c] = s ? a : b;
      }
#pragma unroll
      for (int c = 0; c < R; ++c) {
        const double a = X[k][c], b = X[i][c];
        X[k][c] = s ? b : a;
        X[i][c] = s ? a : b;
      }
    }
    const double piv = A[k][k];
    ok = ok && (piv != 0.0);
    const double r = 1.0 / piv;
#pragma unroll
    for (int i = k + 1; i < n; ++i) {
      const double l = A[i][k] * r;
#pragma unroll
      for (int c = k + 1; c < n; ++c) A[i][c] = fma(-l, A[k][c], A[i][c]);
#pragma unroll
      for (int c = 0; c < R; ++c) X[i][c] = fma(-l, X[k][c], X[i][c]);
    }
  }
  // back substitution
#pragma unroll
  for (int k = n - 1; k >= 0; --k) {
    const double r = 1.0 / A[k][k];
#pragma unroll
    for (int c = 0; c < R; ++c) {
      double s = X[k][c];
#pragma unroll
      for (int j = k + 1; j < n; ++j) s = fma(-A[k][j], X[j][c], s);
      X[k][c] = s * r;
    }
  }
  return ok;
}

// initialize_filter (filter.jl:1-10):
//   β₀ = (I − Φ) \ δ
//   P₀ = vec⁻¹((I − Φ⊗Φ)⁻¹ vec Q), solved on the symmetric subspace: the
//   M(M+1)/2 unknowns P_ij (i ≤ j) of P − ΦPΦ' = Q.  That system is singular iff
//   some λ_iλ_j = 1, exactly when the reference's M²×M² matrix is.
// Returns false where the reference would throw (exact zero pivot).
template <int M, int LEAD>
__device__ __forceinline__ bool init_state(const Params<M, LEAD>& p, double (&beta)[M], double (&P)[M][M]) {
  double A[M][M];
  double x[M][1];
#pragma unroll
  for (int i = 0; i < M; ++i) {
#pragma unroll
    for (int j = 0; j < M; ++j) A[i][j] = (i == j ? 1.0 : 0.0) - p.Phi[i][j];
    x[i][0] = p.delta[i];
  }
  bool ok = gauss_solve<M, 1>(A, x);
#pragma unroll
  for (int i = 0; i < M; ++i) beta[i] = x[i][0];

  constexpr int S = M * (M + 1) / 2;
  double L[S][S];
  double q[S][1];
  int r = 0;
#pragma unroll
  for (int i = 0; i < M; ++i)
#pragma unroll
    for (int j = i; j < M; ++j) {
      int c = 0;
#pragma unroll
      for (int k = 0; k < M; ++k)
#pragma unroll
        for (int l = k; l < M; ++l) {
          // coefficient of P_kl (k ≤ l) in (ΦPΦ')_ij
          double s = p.Phi[i][k] * p.Phi[j][l];
          if (k != l) s = fma(p.Phi[i][l], p.Phi[j][k], s);
          L[r][c] = (r == c ? 1.0 : 0.0) - s;
          ++c;
        }
      q[r][0] = p.Q[i][j];
      ++r;
    }
  ok = gauss_solve<S, 1>(L, q) && ok;
  r = 0;
#pragma unroll
  for (int i = 0; i < M; ++i)
#pragma unroll
    for (int j = i; j < M; ++j) {
      P[i][j] = q[r][0];
      P[j][i] = q[r][0];
      ++r;
    }
  return ok;
}

// Capacitance solve.  With G = Z'Z and B̃ = σ²I + P G (= B' for B = σ²I + G P):
//   W = B̃⁻¹ P = P B⁻¹ (symmetric),  K v = W Z'v,  P_{t|t} = σ² W,
//   v'F⁻¹v = (v'v − u'Wu)/σ²,  det F = σ^{2(N−M)} det B̃.
// Outputs the upper triangle of W and det B̃ (its sign is the sign of det F).
// SYM: return the symmetric part of the computed W (used by the fixed-loading models, whose
// capacitance lanes are exactly those with near-singular Z'Z); otherwise its upper triangle.
template <int M, bool SYM = false>
struct Capacitance {
  __device__ __forceinline__ static void solve(const double (&P)[M][M], const double (&G)[M][M], double sigma2,
                                               double (&W)[M][M], double& det) {
    double A[M][M];
    double X[M][M];
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
      for (int j = 0; j < M; ++j) {
        double s = (i == j) ? sigma2 : 0.0;
#pragma unroll
        for (int l = 0; l < M; ++l) s = fma(P[i][l], G[l][j], s);
        A[i][j] = s;
        X[i][j] = P[i][j];
      }
    // LU with partial pivoting, sign tracked like LAPACK + Julia logabsdet
    double sgn = 1.0;
    double prod = 1.0;
#pragma unroll
    for (int k = 0; k < M; ++k) {
      int p = k;
      double amax = fabs(A[k][k]);
#pragma unroll
      for (int i = k + 1; i < M; ++i) {
        const double a = fabs(A[i][k]);
        const bool gt = a > amax;
        amax = gt ? a : amax;
        p = gt ? i : p;
      }
      sgn = (p != k) ? -sgn : sgn;
#pragma unroll
      for (int i = k + 1; i < M; ++i) {
        const bool s = (p == i);
#pragma unroll
        for (int c = k; c < M; ++c) {
          const double a = A[k][c], b = A[i][c];
          A[k][c] = s ? b : a;
          A[i][c] = s ? a : b;
        }
#pragma unroll
        for (int c = 0; c < M; ++c) {
          const double a = X[k][c], b = X[i][c];
          X[k][c] = s ? b : a;
          X[i][c] = s ? a : b;
        }
      }
      const double piv = A[k][k];
      prod *= piv;
      const double r = 1.0 / piv;
#pragma unroll
      for (int i = k + 1; i < M; ++i) {
        const double l = A[i][k] * r;
#pragma unroll
        for (int c = k + 1; c < M; ++c) A[i][c] = fma(-l, A[k][c], A[i][c]);
#pragma unroll
        for (int c = 0; c < M; ++c) X[i][c] = fma(-l, X[k][c], X[i][c]);
      }
    }
#pragma unroll
    for (int k = M - 1; k >= 0; --k) {
      const double r = 1.0 / A[k][k];
#pragma unroll
      for (int c = 0; c < M; ++c) {
        double s = X[k][c];
#pragma unroll
        for (int j = k + 1; j < M; ++j) s = fma(-A[k][j], X[j][c], s);
        X[k][c] = s * r;
      }
    }
    // W = B̃⁻¹P is symmetric in exact arithmetic; the computed one is not (its asymmetry grows
    // with B̃'s conditioning — measured 7e-9 on the loglik from using one triangle when Z'Z is
    // near-singular).  Use the symmetric part.
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
      for (int j = i; j < M; ++j) W[i][j] = SYM ? 0.5 * (X[i][j] + X[j][i]) : X[i][j];
    det = sgn * prod;
  }
};

// 1/d to ~1 ulp: v_rcp_f64 plus two Newton steps (no IEEE special-casing needed:
// a zero or non-finite d yields a non-finite result, which the callers treat
// exactly like the reference's singular / non-finite cases).
__device__ __forceinline__ double rcp_nr(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  e = fma(-d, r, 1.0);
  return fma(r, e, r);
}

// 1/d from v_rcp_f64 and ONE Newton step (the seed's error squared: ≈ 1 ulp), for the per-step
// LDLᵀ pivots of the fixed-loading filter, where the reciprocal sits on the serial chain
__device__ __forceinline__ double rcp_nr1(double d) {
  const double r = __builtin_amdgcn_rcp(d);
  return fma(r, fma(-d, r, 1.0), r);
}

// Symmetric LDLᵀ (no pivoting) of an M×M matrix S, solving S X = Rhs in place for
// R right-hand sides; returns det S = ∏ d_i (its sign is exact in the factorised
// arithmetic).  Used on S = P + σ²(Z'Z)⁻¹, which is SPD whenever P is PSD.
template <int M, int R>
__device__ __forceinline__ double ldlt_solve(const double (&S)[M][M], double (&X)[M][R]) {
  double L[M][M];  // strictly lower part used
  double a[M][M];  // a[i][k] = L[i][k] * d[k]
  double d[M], rd[M];
#pragma unroll
  for (int j = 0; j < M; ++j) {
    double dj = S[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) dj = fma(-a[j][k], L[j][k], dj);
    d[j] = dj;
    rd[j] = rcp_nr(dj);
#pragma unroll
    for (int i = j + 1; i < M; ++i) {
      double s = S[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) s = fma(-a[i][k], L[j][k], s);
      a[i][j] = s;
      L[i][j] = s * rd[j];
    }
  }
#pragma unroll
  for (int c = 0; c < R; ++c) {
#pragma unroll
    for (int i = 0; i < M; ++i) {
      double s = X[i][c];
#pragma unroll
      for (int k = 0; k < i; ++k) s = fma(-L[i][k], X[k][c], s);
      X[i][c] = s;
    }
#pragma unroll
    for (int i = 0; i < M; ++i) X[i][c] *= rd[i];
#pragma unroll
    for (int i = M - 1; i >= 0; --i) {
      double s = X[i][c];
#pragma unroll
      for (int k = i + 1; k < M; ++k) s = fma(-L[k][i], X[k][c], s);
      X[i][c] = s;
    }
  }
  double det = d[0];
#pragma unroll
  for (int i = 1; i < M; ++i) det *= d[i];
  return det;
}

// The same LDLᵀ split in two, so callers can stream the right-hand sides one at a time
// (fewer live registers; per-element arithmetic identical to ldlt_solve).
template <int M>
struct LDLT {
  double L[M][M];  // strictly lower part used
  double rd[M];    // 1 / d_i
  __device__ __forceinline__ double factor(const double (&S)[M][M]) {
    double a[M][M];
    double d[M];
#pragma unroll
    for (int j = 0; j < M; ++j) {
      double dj = S[j][j];
#pragma unroll
      for (int k = 0; k < j; ++k) dj = fma(-a[j][k], L[j][k], dj);
      d[j] = dj;
      rd[j] = rcp_nr1(dj);
#pragma unroll
      for (int i = j + 1; i < M; ++i) {
        double s = S[i][j];
#pragma unroll
        for (int k = 0; k < j; ++k) s = fma(-a[i][k], L[j][k], s);
        a[i][j] = s;
        L[i][j] = s * rd[j];
      }
    }
    double det = d[0];
#pragma unroll
    for (int i = 1; i < M; ++i) det *= d[i];
    return det;
  }
  __device__ __forceinline__ void solve(double (&x)[M]) const {
#pragma unroll
    for (int i = 0; i < M; ++i) {
      double s = x[i];
#pragma unroll
      for (int k = 0; k < i; ++k) s = fma(-L[i][k], x[k], s);
      x[i] = s;
    }
#pragma unroll
    for (int i = 0; i < M; ++i) x[i] *= rd[i];
#pragma unroll
    for (int i = M - 1; i >= 0; --i) {
      double s = x[i];
#pragma unroll
      for (int k = i + 1; k < M; ++k) s = fma(-L[k][i], x[k], s);
      x[i] = s;
    }
  }
};

// β ← δ + Φ β_{t|t};  P ← Φ P_{t|t} Φ' + Q   (filter.jl:162-176).  Pf: upper triangle.
// `phi(i, j)` returns Φ_ij (registers, or LDS for the 5-factor kernel); each row of Φ is
// read once per product so an LDS-backed Φ costs 2·M² reads per step.
template <int M, class PhiF>
__device__ __forceinline__ void propagate_mean_f(PhiF phi, const double (&delta)[M], const double (&bf)[M],
                                                 double (&beta)[M]) {
#pragma unroll
  for (int i = 0; i < M; ++i) {
    double s = delta[i];
#pragma unroll
    for (int j = 0; j < M; ++j) s = fma(phi(i, j), bf[j], s);
    beta[i] = s;
  }
}

template <int M, class PhiF>
__device__ __forceinline__ void propagate_cov_f(PhiF phi, const double (&Q)[M][M], const double (&Pf)[M][M],
                                                double (&Pm)[M][M]) {
  double A[M][M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    double f[M];
#pragma unroll
    for (int j = 0; j < M; ++j) f[j] = phi(i, j);
#pragma unroll
    for (int j = 0; j < M; ++j) {
      double a = 0.0;
#pragma unroll
      for (int l = 0; l < M; ++l) a = fma(f[l], (l <= j) ? Pf[l][j] : Pf[j][l], a);
      A[i][j] = a;
    }
  }
#pragma unroll
  for (int j = 0; j < M; ++j) {
    double f[M];
#pragma unroll
    for (int l = 0; l < M; ++l) f[l] = phi(j, l);
#pragma unroll
    for (int i = 0; i <= j; ++i) {
      double s = Q[i][j];
#pragma unroll
      for (int l = 0; l < M; ++l) s = fma(A[i][l], f[l], s);
      Pm[i][j] = s;
      Pm[j][i] = s;
    }
  }
}

template <int M, class PhiF>
__device__ __forceinline__ void propagate_state_f(PhiF phi, const double (&Q)[M][M], const double (&delta)[M],
                                                  const double (&bf)[M], const double (&Pf)[M][M], double (&beta)[M],
                                                  double (&Pm)[M][M]) {
  propagate_mean_f<M>(phi, delta, bf, beta);
  propagate_cov_f<M>(phi, Q, Pf, Pm);
}

template <int M, int LEAD>
__device__ __forceinline__ void propagate_state(const Params<M, LEAD>& p, const double (&bf)[M], const double (&Pf)[M][M],
                                                double (&beta)[M], double (&Pm)[M][M]) {
  propagate_state_f<M>([&](int i, int j) { return p.Phi[i][j]; }, p.Q, p.delta, bf, Pf, beta, Pm);
}

// x + (x of the partner lane) for the butterfly level `lvl` (partner distance 2^lvl,
// every partner inside the same aligned group of 2^(lvl+1) lanes).
template <int LVL>
__device__ __forceinline__ double group_level_sum(double x) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  if constexpr (LVL == 0 || LVL == 1 || LVL == 2 || LVL == 3) {
    // quad_perm xor1 / xor2, row_half_mirror, row_mirror
    constexpr int ctrl = LVL == 0 ? 0xB1 : LVL == 1 ? 0x4E : LVL == 2 ? 0x141 : 0x140;
    const int plo = __builtin_amdgcn_mov_dpp(lo, ctrl, 0xf, 0xf, true);
    const int phi = __builtin_amdgcn_mov_dpp(hi, ctrl, 0xf, 0xf, true);
    return x + __hiloint2double(phi, plo);
  } else if constexpr (LVL == 4) {
    // rows (0,1), (2,3): vdst' = [r0 r0 r2 r2], src' = [r1 r1 r3 r3]
    const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return __hiloint2double(rh[0], rl[0]) + __hiloint2double(rh[1], rl[1]);
  } else {
    // halves: vdst' = [lo lo], src' = [hi hi]
    const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return __hiloint2double(rh[0], rl[0]) + __hiloint2double(rh[1], rl[1]);
  }
}

// The value of role S (lane & 3 = S) of this lane's quad: DPP quad_perm broadcast.  Used by the
// TVλ filters to distribute their 4×4 update over the four roles of each quad.
template <int S>
__device__ __forceinline__ double quad_bcast_f64(double x) {
  constexpr int ctrl = S | (S << 2) | (S << 4) | (S << 6);
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), ctrl, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), ctrl, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
// the value held by role qr ^ R of this lane's quad (R = 1, 2, 3)
template <int R>
__device__ __forceinline__ double quad_xor_f64(double x) {
  constexpr int ctrl = (0 ^ R) | ((1 ^ R) << 2) | ((2 ^ R) << 4) | ((3 ^ R) << 6);
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), ctrl, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), ctrl, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
// v[i] for a lane-dependent i in [0, 4): a two-level mux on the bits of i (a chain of i == k selects is turned
// into a scratch-indexed load by the compiler)
__device__ __forceinline__ double sel4_f64(const double (&v)[4], int i) {
  const bool b0 = (i & 1) != 0, b1 = (i & 2) != 0;
  const double lo = b0 ? v[1] : v[0];
  const double hi = b0 ? v[3] : v[2];
  return b1 ? hi : lo;
}
// Column qr of the symmetric 4×4 whose role k holds the upper entries v[i], i ≤ k, of its column: col[k] = v[k] for
// k ≤ qr and role k's v[qr] below the diagonal — the quad transpose done with DPP alone (role qr ^ d hands over its
// v[qr] at distance d), no LDS round trip.  The same values as the LDS exchange, bit for bit.
__device__ __forceinline__ void quad_mirror_f64(int qr, const double (&v)[4], double (&col)[4]) {
  const double r1 = quad_xor_f64<1>(sel4_f64(v, qr ^ 1));
  const double r2 = quad_xor_f64<2>(sel4_f64(v, qr ^ 2));
  const double r3 = quad_xor_f64<3>(sel4_f64(v, qr ^ 3));
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int d = k ^ qr;  // bit mux, as sel4_f64
    const bool b0 = (d & 1) != 0, b1 = (d & 2) != 0;
    const double o = b1 ? (b0 ? r3 : r2) : r1;
    col[k] = k <= qr ? v[k] : o;
  }
}
// rows of a 4×4 whose row S lives in role S, into every lane
template <int M>
__device__ __forceinline__ void quad_gather_rows(const double (&row)[M], double (&X)[M][M]) {
  static_assert(M == 4, "quad roles hold the rows of a 4×4");
#pragma unroll
  for (int k = 0; k < M; ++k) {
    X[0][k] = quad_bcast_f64<0>(row[k]);
    X[1][k] = quad_bcast_f64<1>(row[k]);
    X[2][k] = quad_bcast_f64<2>(row[k]);
    X[3][k] = quad_bcast_f64<3>(row[k]);
  }
}
// LDS writes of this wave visible to its own later LDS reads
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Sum over the aligned group of L lanes (DPP / permlane butterflies, no LDS); every lane of
// the group receives the total.
template <int L>
__device__ __forceinline__ double group_sum(double x) {
  if constexpr (L >= 2) x = group_level_sum<0>(x);
  if constexpr (L >= 4) x = group_level_sum<1>(x);
  if constexpr (L >= 8) x = group_level_sum<2>(x);
  if constexpr (L >= 16) x = group_level_sum<3>(x);
  if constexpr (L >= 32) x = group_level_sum<4>(x);
  if constexpr (L >= 64) x = group_level_sum<5>(x);
  return x;
}

// log|∏ d_t| accumulated as mantissa × 2^expo: one multiply and two frexp
// instructions per step instead of a software FP64 log.
struct LogDetAcc {
  double mant = 1.0;
  int expo = 0;
  __device__ __forceinline__ void mul(double d) {
    const double m = mant * fabs(d);
    expo += __builtin_amdgcn_frexp_exp(m);
    mant = __builtin_amdgcn_frexp_mant(m);
  }
  __device__ __forceinline__ double log_value() const { return log(mant) + (double)expo * kLn2; }
};

}  // namespace yfm

// yfm_fixedz.hpp — the per-candidate filter of the fixed-loading models (DNS, GNS5),
// shared by the one-filter-per-lane kernel (yfm_kernels.hip) and the one-filter-per-lane-
// group kernel for large maturity counts (yfm_group.hip).  The kernels only differ in how
// they form z̃_t = Z'ỹ_t (MFMA tiles, VALU dot products, or a lane-group reduction).
//
// Restates filter.jl:125-179 (filter!), :182-209 (get_loss) and :1-10 (initialize_filter)
// in the collapsed form of DESIGN.md §3.1 (see yfm_kernels.hip's header).
#pragma once
// No implicit FMA contraction in the fixed-loading kernels: every fused multiply-add is an
// explicit fma(), so the kernels that share this code (the per-lane and the lane-group
// kernel) round identically wherever it is inlined, whatever the surrounding code.
#pragma clang fp contract(off)
#include "yfm_device.hpp"

namespace yfm {

// The collapsed-form measurement update in two halves:
//   covariance (data-independent): S = P + R, its LDLᵀ and det S, P_{t|t} = P S⁻¹R;
//   mean: ĉ, the residual ‖ỹ − Zĉ‖², c = ĉ − β, x = S⁻¹c, q = v'F⁻¹v, β_{t|t} = β + P x.
// collapsed_update runs both in one lane; the two-wave DNS kernel (yfm_split.hip) runs them on
// different waves, the mean wave reading (L, 1/d, P, det S) from the covariance wave.  Each value
// has the same expression in both, so the two kernels give the same bits.
template <int M>
__device__ __forceinline__ double collapsed_cov(const double (&R)[M][M], const double (&Pm)[M][M], LDLT<M>& f,
                                                double (&Pf)[M][M]) {
  double S[M][M];
#pragma unroll
  for (int i = 0; i < M; ++i)
#pragma unroll
    for (int j = 0; j <= i; ++j) S[i][j] = Pm[i][j] + R[i][j];  // LDLᵀ reads the lower triangle only
  const double det = f.factor(S);
  // right-hand sides streamed one at a time: S⁻¹R column by column
#pragma unroll
  for (int j = 0; j < M; ++j) {
    double xj[M];
#pragma unroll
    for (int i = 0; i < M; ++i) xj[i] = R[i][j];
    f.solve(xj);
#pragma unroll
    for (int i = 0; i <= j; ++i) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < M; ++k) s = fma(Pm[i][k], xj[k], s);
      Pf[i][j] = s;
    }
  }
  return det;
}

template <int M>
__device__ __forceinline__ void collapsed_mean(const double (&zt)[M - 1], double ybar, double ytt, const double (&R)[M][M],
                                               double rsig2, const double (&beta)[M], const double (&Pm)[M][M],
                                               const LDLT<M>& f, double (&bf)[M], double& q) {
  double zs[M - 1];
#pragma unroll
  for (int j = 0; j < M - 1; ++j) zs[j] = zt[j] * rsig2;
  double ch[M];  // ĉ = G⁻¹(0, z̃) (= R/σ² · (0, z̃))
#pragma unroll
  for (int i = 0; i < M; ++i) {
    double s = 0.0;
#pragma unroll
    for (int j = 1; j < M; ++j) s = fma(R[i][j], zs[j - 1], s);
    ch[i] = s;
  }
  double rr = ytt;  // ‖ỹ − Zĉ‖² = ỹ'ỹ − z̃'ĉ
#pragma unroll
  for (int j = 1; j < M; ++j) rr = fma(-zt[j - 1], ch[j], rr);
  ch[0] += ybar;
  double c[M], x[M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    c[i] = ch[i] - beta[i];
    x[i] = c[i];
  }
  f.solve(x);  // x = S⁻¹c
  double cx = 0.0;
#pragma unroll
  for (int i = 0; i < M; ++i) cx = fma(c[i], x[i], cx);
  q = fma(rr, rsig2, cx);
#pragma unroll
  for (int i = 0; i < M; ++i) {
    double s = beta[i];
#pragma unroll
    for (int k = 0; k < M; ++k) s = fma(Pm[i][k], x[k], s);
    bf[i] = s;
  }
}

// Collapsed-form measurement update (see the header): returns det S and q = v'F⁻¹v,
// writes β_{t|t} (bf) and the upper triangle of P_{t|t} (Pf).  The same arithmetic as
// collapsed_cov + collapsed_mean, as one body (the per-lane kernels keep this form).
template <int M>
__device__ __forceinline__ void collapsed_update(const double (&zt)[M - 1], double ybar, double ytt,
                                                 const double (&R)[M][M], double rsig2, const double (&beta)[M],
                                                 const double (&Pm)[M][M], double (&bf)[M], double (&Pf)[M][M],
                                                 double& det, double& q) {
  double zs[M - 1];
#pragma unroll
  for (int j = 0; j < M - 1; ++j) zs[j] = zt[j] * rsig2;
  double ch[M];  // ĉ = G⁻¹(0, z̃) (= R/σ² · (0, z̃))
#pragma unroll
  for (int i = 0; i < M; ++i) {
    double s = 0.0;
#pragma unroll
    for (int j = 1; j < M; ++j) s = fma(R[i][j], zs[j - 1], s);
    ch[i] = s;
  }
  double rr = ytt;  // ‖ỹ − Zĉ‖² = ỹ'ỹ − z̃'ĉ
#pragma unroll
  for (int j = 1; j < M; ++j) rr = fma(-zt[j - 1], ch[j], rr);
  ch[0] += ybar;
  double S[M][M];
  double c[M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    c[i] = ch[i] - beta[i];
#pragma unroll
    for (int j = 0; j <= i; ++j) S[i][j] = Pm[i][j] + R[i][j];  // LDLᵀ reads the lower triangle only
  }
  LDLT<M> f;
  det = f.factor(S);
  // right-hand sides streamed one at a time: x = S⁻¹c, then S⁻¹R column by column
  double x[M];
#pragma unroll
  for (int i = 0; i < M; ++i) x[i] = c[i];
  f.solve(x);
  double cx = 0.0;
#pragma unroll
  for (int i = 0; i < M; ++i) cx = fma(c[i], x[i], cx);
  q = fma(rr, rsig2, cx);
#pragma unroll
  for (int i = 0; i < M; ++i) {
    double s = beta[i];
#pragma unroll
    for (int k = 0; k < M; ++k) s = fma(Pm[i][k], x[k], s);
    bf[i] = s;
  }
#pragma unroll
  for (int j = 0; j < M; ++j) {
    double xj[M];
#pragma unroll
    for (int i = 0; i < M; ++i) xj[i] = R[i][j];
    f.solve(xj);
#pragma unroll
    for (int i = 0; i <= j; ++i) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < M; ++k) s = fma(Pm[i][k], xj[k], s);
      Pf[i][j] = s;
    }
  }
}


// Lanes whose Z'Z is ill-conditioned (κ₁ ≥ kCollapsedKappa), singular, or has fewer maturities than
// states are not evaluated here: the kernels append them to a deferral list and the double-double
// capacitance kernel (yfm_fixedz_dd.hip) evaluates them afterwards.
//
// The collapsed form's rounding grows with κ(Z'Z) through R = σ²(Z'Z)⁻¹ and ĉ = (Z'Z)⁻¹Z'y
// (measured: up to ≈ κ·3e-17 relative on the loglik, e.g. 1.8e-9 at κ₁ = 5e7 on a 40-step
// GNS5 panel, where the reference's dense path is 1e-13 from exact).  κ₁ is ≈ 400 for DNS on the
// usual grids and 2.5e4 … 7.0e5 over the 1,048,576 GNS5 candidates of config 5, so at 1e6 no
// benchmark lane is deferred while the error of every collapsed lane stays ≲ 3e-11.
constexpr double kCollapsedKappa = 1e6;

// P ← Φ P_{t|t} Φ' + Q as propagate_cov_f (bitwise), except that a frozen lane keeps its P; returns the
// largest change of an entry and the largest new entry (the freeze test of FixedZFilter)
template <int M, int LEAD>
__device__ __forceinline__ void propagate_cov_freeze(const Params<M, LEAD>& p, const double (&Pf)[M][M],
                                                     double (&Pm)[M][M], bool frozen, double& dmax, double& nmax) {
  double A[M][M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
#pragma unroll
    for (int j = 0; j < M; ++j) {
      double a = 0.0;
#pragma unroll
      for (int l = 0; l < M; ++l) a = fma(p.Phi[i][l], (l <= j) ? Pf[l][j] : Pf[j][l], a);
      A[i][j] = a;
    }
  }
  dmax = 0.0;
  nmax = 0.0;
#pragma unroll
  for (int j = 0; j < M; ++j) {
#pragma unroll
    for (int i = 0; i <= j; ++i) {
      double t = p.Q[i][j];
#pragma unroll
      for (int l = 0; l < M; ++l) t = fma(A[i][l], p.Phi[j][l], t);
      dmax = fmax(dmax, fabs(t - Pm[i][j]));
      nmax = fmax(nmax, fabs(t));
      const double v = frozen ? Pm[i][j] : t;
      Pm[i][j] = v;
      Pm[j][i] = v;
    }
  }
}

// Upper bound of C = Σ_{k≥1} ‖A^k‖_∞² for the closed-loop matrix A = Φ(I − KZ) = Φ R S⁻¹, S = P + R
// (I − KZ = I − P S⁻¹ = R S⁻¹ in the collapsed form; ‖·‖_∞ = largest absolute row sum).  The Riccati
// differences δ_t = P_{t+1} − P_t obey the exact identity δ_{t+1} = A_{t+1} δ_t A_t' (information form:
// f(P₁) − f(P₂) = Φ(I + P₁J)⁻¹(P₁ − P₂)(I + JP₂)⁻¹Φ', J = Z'Z/σ²), and |(A δ A')_ij| ≤ ‖δ‖_max
// Σ_k|A_ik| Σ_l|A_jl|, so once the A_t agree with A to first order the drift still to come after a step
// that moved P by δ is ‖Σ_{k≥1} δ_{t+k}‖_max ≤ C ‖δ‖_max — whatever the eigenvalues of A (real or
// complex, monotone or oscillating convergence).  From A … A⁴ by sub-multiplicativity:
// C ≤ (‖A‖² + ‖A²‖² + ‖A³‖² + ‖A⁴‖²)/(1 − ‖A⁴‖²); +Inf when ‖A⁴‖_∞ ≥ 1 (no bound: never frozen early).
//
// The loglik's sensitivity (round 5; the de-aliased sweep's case 9: a 1.3e-11 loglik change).  Within 2^-52 of
// the full recursion's P is not enough by itself: a frozen P that differs from it by ΔP changes each innovation
// term c'S⁻¹c by c'S⁻¹ΔP S⁻¹c, i.e. relatively by up to ‖ΔP‖‖S⁻¹‖ ≈ 2^-52·‖P‖‖S⁻¹‖, and the filtered mean
// carries the gain change ΔK = R S⁻¹ΔP S⁻¹ through the closed loop, ‖Δβ_t‖ ≤ C₁‖ΔK‖ max‖c‖ with
// C₁ = Σ_{k≥1} ‖A^k‖_∞ ≤ (‖A‖ + ‖A²‖ + ‖A³‖ + ‖A⁴‖)/(1 − ‖A⁴‖).  A lane is allowed to freeze short of a bitwise
// fixed point only when g = max(1, C₁)·‖P‖_∞‖S⁻¹‖_∞ ≤ kLoglikGainCap (else C = +Inf: d = 0 only), which keeps
// the relative loglik change near 512·2^-52 ≈ 1e-13 unless the loglik itself cancels.  Calibrated with the CPU
// model of the rule (tools/steady_rule.py --rules gain): the case-9 class 6.8e-12 → 1.8e-14; the config-2
// class (g ≤ 22) keeps every freeze; θ₀ ± 0.3 has 0.1% of its lanes above the cap.
// Row j of A^k is (A')^k e_j, A'v = S⁻¹(R(Φ'v)): no M×M temporaries beyond the factors of S (the
// GNS5 kernel has no registers for A and its powers; M ≤ 3 runs the M start vectors side by side).
constexpr double kLoglikGainCap = 512.0;

template <int M, int LEAD>
__device__ __forceinline__ double contraction_bound(const Params<M, LEAD>& p, const double (&R)[M][M],
                                                    const double (&Pm)[M][M]) {
  double S[M][M];
#pragma unroll
  for (int i = 0; i < M; ++i)
#pragma unroll
    for (int j = 0; j <= i; ++j) S[i][j] = Pm[i][j] + R[i][j];
  LDLT<M> f;
  (void)f.factor(S);
  double n[4] = {0.0, 0.0, 0.0, 0.0};  // ‖A^k‖_∞, k = 1..4
  double sinv = 0.0;                   // ‖S⁻¹‖_∞ (S⁻¹ symmetric: the largest column sum of |S⁻¹ e_j|)
  // one row of A^k per start vector e_j: v ← S⁻¹R Φ'v, ‖A^k‖_∞ = max_j Σ_i |v_i|
  auto power_step = [&](double (&v)[M]) {
    double w[M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
      double s = 0.0;
#pragma unroll
      for (int l = 0; l < M; ++l) s = fma(p.Phi[l][i], v[l], s);  // Φ'v
      w[i] = s;
    }
#pragma unroll
    for (int i = 0; i < M; ++i) {
      double s = 0.0;
#pragma unroll
      for (int l = 0; l < M; ++l) s = fma(R[i][l], w[l], s);  // R Φ'v
      v[i] = s;
    }
    f.solve(v);  // S⁻¹ R Φ'v
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < M; ++i) sum += fabs(v[i]);
    return sum;
  };
  auto sinv_col = [&](int j) {  // Σ_i |(S⁻¹ e_j)_i|
    double v[M];
#pragma unroll
    for (int i = 0; i < M; ++i) v[i] = (i == j) ? 1.0 : 0.0;
    f.solve(v);
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < M; ++i) sum += fabs(v[i]);
    return sum;
  };
  if constexpr (M <= 3) {
    // the M start vectors side by side: M independent chains per power (the rolled form below is one
    // serial chain of 4M solves, ≈ 3 µs of a config-2 launch; profiles/r4/exp1/)
    double V[M][M];
#pragma unroll
    for (int j = 0; j < M; ++j)
#pragma unroll
      for (int i = 0; i < M; ++i) V[j][i] = (i == j) ? 1.0 : 0.0;
#pragma unroll
    for (int j = 0; j < M; ++j) sinv = fmax(sinv, sinv_col(j));
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int j = 0; j < M; ++j) n[k] = fmax(n[k], power_step(V[j]));
  } else {
    // (GNS5: one column and one power at a time keeps the temporaries to two M-vectors)
#pragma unroll 1
    for (int j = 0; j < M; ++j) {
      sinv = fmax(sinv, sinv_col(j));
      double v[M];
#pragma unroll
      for (int i = 0; i < M; ++i) v[i] = (i == j) ? 1.0 : 0.0;
#pragma unroll 1
      for (int k = 0; k < 4; ++k) {
        const double sum = power_step(v);
        n[0] = (k == 0) ? fmax(n[0], sum) : n[0];
        n[1] = (k == 1) ? fmax(n[1], sum) : n[1];
        n[2] = (k == 2) ? fmax(n[2], sum) : n[2];
        n[3] = (k == 3) ? fmax(n[3], sum) : n[3];
      }
    }
  }
  double pn = 0.0;  // ‖P‖_∞
#pragma unroll
  for (int i = 0; i < M; ++i) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < M; ++j) s += fabs(Pm[i][j]);
    pn = fmax(pn, s);
  }
  const double n0 = n[0], n1 = n[1], n2 = n[2], n3 = n[3];
  const double q = n3 * n3;
  // rounding of the bounds themselves: a few ulps; the 1.01 margins cover it
  const double c1 = 1.01 * (n0 + n1 + n2 + n3) / (1.0 - n3);
  const bool ok = (q < 1.0) && (fmax(1.0, c1) * pn * sinv <= kLoglikGainCap);
  return ok ? 1.01 * (n0 * n0 + n1 * n1 + n2 * n2 + q) / (1.0 - q) : __builtin_inf();
}

template <int M, int LEAD, bool RECORD, bool STEADY = false, bool SPLIT_FORM = false>
struct FixedZFilter {
  Params<M, LEAD> p;
  double sigma2, rsig2;
  double R[M][M];  // σ²(Z'Z)⁻¹ (meaningful on collapsed lanes only)
  double logdetG = 0.0;
  bool collapsed = false, init_ok = false;
  int N = 0;
  double beta[M], Pm[M][M];
  LogDetAcc ld;
  double sumq = 0.0;
  bool neg = false;
  double last_det = 0.0, last_q = 0.0;  // fresh model: F = 0, F⁻¹ = 0, v = 0 (kalmanbasemodel.jl:65-67)

  // ---- frozen covariance (STEADY: loglik mode of the per-lane kernel) ----
  // With Z fixed the covariance recursion P ↦ Φ P(P + R)⁻¹R Φ' + Q does not depend on the data and
  // converges to the Riccati fixed point.  A lane freezes its P after a data step that moved it by a
  // relative d (largest entry change / largest entry) when
  //   d = 0 — a bitwise fixed point of the FP64 recursion, which the full recursion never leaves, or
  //   d ≤ 2^-46 and d·C ≤ 2^-52 — C bounds Σ_{k≥1}‖A^k‖_∞² for the lane's closed-loop matrix
  //   A = Φ R S⁻¹ (contraction_bound, computed once, prepare_bound), so every later P of the
  //   full recursion is within 2^-52 (relative to its largest entry, to first order in d) of the frozen
  //   one — inside the FP64 recursion's own rounding jitter — for monotone and oscillating
  //   (complex-eigenvalue) convergence alike (DESIGN.md §3.1 carries the bound on the loglik); and the
  //   loglik's sensitivity max(1, C₁)‖P‖‖S⁻¹‖ ≤ 512 (contraction_bound: else only d = 0 freezes);
  // a frozen lane keeps P (and so S = P + R and its factors) for every later data step, until a
  // prediction-only step (a NaN column) moves P.  The freeze step depends on the lane's θ alone, so its
  // loglik does not depend on the batch.  Once EVERY lane of a wave is frozen the wave runs the mean
  // update only, with the factors of S cached — bitwise the full step's values for a frozen lane (the
  // same S, factorised by the same code).
  // M ≤ 3 caches the factors of S at the wave's freeze; M = 5 has no registers for them (the GNS5
  // kernel uses the whole file) and refactors the constant S every steady step instead, so only the
  // covariance half (P S⁻¹R, ΦPΦ' + Q) is skipped — bitwise the same values either way
  static constexpr bool kCacheFactors = (M <= 3);
  bool steady_ok = false;    // the runtime switch (YFM_DNS_STEADY, default on)
  bool frozen = false;
  double cbound = -1.0;      // 2·C of contraction_bound (< 0: not computed yet)
  double dlast = __builtin_inf();  // d of the lane's last data step before its freeze
  bool wave_frozen = false;  // wave-uniform at every block boundary (wave_freeze)
  LDLT<M> fs;                // factors of S = P + R at the frozen P (valid while wave_frozen)
  double dets = 0.0;
  // A frozen lane's det S is the same number at every data step (the same S, factorised by the same
  // code), so its log-det terms are counted instead of multiplied into `ld` one by one: nfz frozen data
  // steps of det fzdet since the freeze, folded into fzlog (Σ n·log|det|) when the lane thaws and at the
  // end.  Every frozen data step counts, whichever loop (steady or full) ran it, so the loglik stays
  // independent of the batch; the steady loop adds its block's steps in one go (count_steady).
  int nfz = 0;
  double fzdet = 1.0, fzlog = 0.0;
  __device__ __forceinline__ void count_frozen(double det) {
    fzdet = nfz == 0 ? det : fzdet;
    ++nfz;
  }
  __device__ __forceinline__ void fold_frozen() {
    fzlog += nfz == 0 ? 0.0 : (double)nfz * log(fabs(fzdet));
    neg = neg || (nfz != 0 && fzdet < 0.0);
    nfz = 0;
  }
  __device__ __forceinline__ void count_steady(int steps) { nfz += steps; }

  // the freeze test after a data step that moved P by (dmax, nmax); Pm holds the new P
  __device__ __forceinline__ void freeze_test(double dmax, double nmax) {
    const double d = dmax / nmax;
    dlast = frozen ? dlast : d;
    const bool ok = (d == 0.0) || (d <= 0x1p-46 && cbound >= 0.0 && d * cbound <= 0x1p-52);
    frozen = frozen || (ok && steady_ok);
  }
  // C of contraction_bound, once per lane, at a block boundary (outside the unrolled steps: its
  // temporaries would otherwise coexist with two steps' operands), as soon as the lane's P has
  // converged to 2^-26: A then agrees with the fixed point's closed loop to ≈ κ(S)·2^-26, and the
  // factor 2 on C covers that
  __device__ __forceinline__ void prepare_bound() {
    if (cbound < 0.0 && steady_ok && dlast <= 0x1p-26) cbound = 2.0 * contraction_bound<M, LEAD>(p, R, Pm);
  }
  // a prediction-only step moves P: the lane thaws (and clears the wave's state at the block's vote)
  __device__ __forceinline__ void thaw() {
    fold_frozen();
    frozen = false;
    wave_frozen = false;
  }
  // wave vote at the end of every full block (every lane of the wave calls this at the same point):
  // `part` = the lane's result counts.  A lane that thawed during the block (a NaN column inside its
  // window) clears the state for the whole wave, so wave_frozen is wave-uniform again — lanes outside
  // their windows (or past B, mirroring candidate B − 1) never thaw and must not keep it alone.
  __device__ __forceinline__ void wave_freeze(bool part) {
    wave_frozen = __all(wave_frozen);
    if (wave_frozen) return;
    if (__all(frozen || !part)) {
      if constexpr (kCacheFactors) {
        double S[M][M];
#pragma unroll
        for (int i = 0; i < M; ++i)
#pragma unroll
          for (int j = 0; j <= i; ++j) S[i][j] = Pm[i][j] + R[i][j];
        dets = fs.factor(S);
        fzdet = nfz == 0 ? dets : fzdet;  // a lane whose first frozen data step is a steady one
      }
      wave_frozen = true;
    }
  }
  // one data step of a frozen wave: the mean update of collapsed_update with the cached factors (its
  // log-det term is counted by the caller's count_steady)
  __device__ __forceinline__ void steady_step(const double (&zc)[M - 1], double2 yb_c) {
    double bf[M], q, det;
    if constexpr (kCacheFactors) {
      collapsed_mean<M>(zc, yb_c.x, yb_c.y, R, rsig2, beta, Pm, fs, bf, q);
      det = dets;
    } else {
      double S[M][M];
#pragma unroll
      for (int i = 0; i < M; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) S[i][j] = Pm[i][j] + R[i][j];
      LDLT<M> fl;
      det = fl.factor(S);
      collapsed_mean<M>(zc, yb_c.x, yb_c.y, R, rsig2, beta, Pm, fl, bf, q);
    }
    propagate_mean_f<M>([&](int i, int j) { return p.Phi[i][j]; }, p.delta, bf, beta);
    last_det = det;
    last_q = q;
    if constexpr (!kCacheFactors) fzdet = nfz == 0 ? det : fzdet;  // (M = 5 refactors S: the same bits)
    sumq += q;
  }

  // G = Z'Z → R, log det G, collapsed or deferred; then initialize_filter.
  // do_init = false: the caller loads the initial state itself (fixedz_init_kernel's record)
  __device__ __forceinline__ void setup(const double (&G)[M][M], int N_, bool do_init = true) {
    N = N_;
    sigma2 = p.sigma2;
    rsig2 = 1.0 / sigma2;
    double A[M][M], X[M][M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
#pragma unroll
      for (int j = 0; j < M; ++j) {
        A[i][j] = G[i][j];
        X[i][j] = (i == j) ? 1.0 : 0.0;
      }
    }
    const bool ok = gauss_solve<M, M>(A, X);
    double detG = 1.0;
#pragma unroll
    for (int i = 0; i < M; ++i) detG *= A[i][i];
    detG = fabs(detG);
    double nG = 0.0, nX = 0.0;  // κ₁ = ‖G‖₁‖G⁻¹‖₁
#pragma unroll
    for (int j = 0; j < M; ++j) {
      double cg = 0.0, cx = 0.0;
#pragma unroll
      for (int i = 0; i < M; ++i) {
        cg += fabs(G[i][j]);
        cx += fabs(X[i][j]);
      }
      nG = fmax(nG, cg);
      nX = fmax(nX, cx);
    }
    collapsed = ok && (N >= M) && (nG * nX < kCollapsedKappa);
    logdetG = collapsed ? log(detG) : 0.0;
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
      for (int j = 0; j < M; ++j) R[i][j] = sigma2 * 0.5 * (X[i][j] + X[j][i]);
    if (do_init) init_ok = init_state<M, LEAD>(p, beta, Pm);
  }

  __device__ __forceinline__ void update(const double (&zc)[M - 1], double2 yb_c, double (&bf)[M], double (&Pf)[M][M],
                                         double& det, double& q) const {
    if constexpr (SPLIT_FORM) {
      LDLT<M> fl;
      det = collapsed_cov<M>(R, Pm, fl, Pf);
      collapsed_mean<M>(zc, yb_c.x, yb_c.y, R, rsig2, beta, Pm, fl, bf, q);
    } else {
      collapsed_update<M>(zc, yb_c.x, yb_c.y, R, rsig2, beta, Pm, bf, Pf, det, q);
    }
  }

  // One filter! call on column t given z̃_t (zc), (ȳ, ỹ'ỹ) = yb and (nan flag, y'y) = meta.
  // `fast`: the caller guarantees t ≥ 1, a data column and an active lane (no masking).
  __device__ __forceinline__ void step(int t, const double (&zc)[M - 1], double2 yb_c, double2 meta_c, bool fast,
                                       int my_steps, int my_data) {
    if (fast) {
      double bf[M], Pf[M][M], det, q;
      update(zc, yb_c, bf, Pf, det, q);
      // (a singular F at t ≥ 2 makes the loglik −Inf whatever the state; trajectories skip the update)
      if constexpr (STEADY) {
        // (the log-det term first: `frozen` as it stood for this step's S)
        if (frozen) {
          count_frozen(det);
        } else {
          ld.mul(det);
          neg = neg || (det < 0.0);
        }
        propagate_mean_f<M>([&](int i, int j) { return p.Phi[i][j]; }, p.delta, bf, beta);
        double dmax, nmax;
        propagate_cov_freeze<M, LEAD>(p, Pf, Pm, frozen, dmax, nmax);
        freeze_test(dmax, nmax);
      } else {
        if (!RECORD || det != 0.0) propagate_state<M, LEAD>(p, bf, Pf, beta, Pm);
        ld.mul(det);
        neg = neg || (det < 0.0);
      }
      last_det = det;
      last_q = q;
      sumq += q;
      return;
    }
    const bool act = t < my_steps;
    const bool acc = t >= 1;  // Julia t > 1 (filter.jl:194)
    if (!act) return;
    if (meta_c.x != 0.0 || t >= my_data) {
      // NaN column: prediction only (filter.jl:126-140); F, v stale → the loglik
      // re-adds the previous term (filter.jl:195 reads base.F / base.v unchanged).
      double Pf[M][M];
#pragma unroll
      for (int i = 0; i < M; ++i)
#pragma unroll
        for (int j = i; j < M; ++j) Pf[i][j] = Pm[i][j];
      double bf[M];
#pragma unroll
      for (int i = 0; i < M; ++i) bf[i] = beta[i];
      propagate_state<M, LEAD>(p, bf, Pf, beta, Pm);
      if constexpr (STEADY) thaw();
      if (acc) {
        ld.mul(last_det);
        sumq += last_q;
        neg = neg || (last_det < 0.0);
      }
      return;
    }
    double det, q;
    double bf[M];
    double Pf[M][M];
    update(zc, yb_c, bf, Pf, det, q);
    const bool upd = det != 0.0;  // inv(F) threw: return without the update (filter.jl:151-154)
    const bool was_frozen = frozen;
    if constexpr (STEADY) {
      if (upd) {
        propagate_mean_f<M>([&](int i, int j) { return p.Phi[i][j]; }, p.delta, bf, beta);
        double dmax, nmax;
        propagate_cov_freeze<M, LEAD>(p, Pf, Pm, frozen, dmax, nmax);
        freeze_test(dmax, nmax);
      }
    } else if (upd) {
      propagate_state<M, LEAD>(p, bf, Pf, beta, Pm);
    }
    last_det = det;
    last_q = upd ? q : __builtin_nan("");
    if (acc) {
      if (STEADY && was_frozen) {
        count_frozen(det);
      } else {
        ld.mul(det);
        neg = neg || (det < 0.0);
      }
      sumq += last_q;
    }
  }

  // the state after step t into slot t − max(0, my_steps − rec_len) (the last rec_len steps)
  __device__ __forceinline__ void record(int t, int b, int my_steps, int rec_len, double* __restrict__ rec_beta,
                                         double* __restrict__ rec_P) const {
    const int slot = t - max(0, my_steps - rec_len);
    if (t < my_steps && slot >= 0) {
      const size_t o = (size_t)b * (size_t)rec_len + slot;
#pragma unroll
      for (int i = 0; i < M; ++i) rec_beta[o * M + i] = beta[i];
      if (rec_P) {
#pragma unroll
        for (int j = 0; j < M; ++j)
#pragma unroll
          for (int i = 0; i < M; ++i) rec_P[o * M * M + j * M + i] = Pm[i][j];
      }
    }
  }

  // get_loss's result (filter.jl:182-209); NaN + flag where initialize_filter throws
  __device__ __forceinline__ double loglik(int nobs, unsigned int* __restrict__ flags) const {
    double ll;
    if (!init_ok) {
      ll = __builtin_nan("");  // the reference throws from initialize_filter
      atomicAdd(&flags[0], 1u);
    } else {
      const int nterms = max(nobs - 2, 0);
      if (nterms == 0) {
        ll = 0.0;
      } else {
        const double per_term = (double)(N - M) * log(sigma2) + logdetG + (double)N * kLog2Pi;
        double lf = 0.0;  // the frozen steps' log-det terms (STEADY)
        if constexpr (STEADY) lf = fzlog + (nfz == 0 ? 0.0 : (double)nfz * log(fabs(fzdet)));
        ll = -0.5 * ((double)nterms * per_term + (ld.log_value() + lf) + sumq);
      }
      const bool fneg = STEADY && nfz != 0 && fzdet < 0.0;
      if (neg || fneg || !isfinite(ll)) {  // DomainError / non-finite → -Inf (filter.jl:197-204)
        ll = -__builtin_inf();
        atomicAdd(&flags[1], 1u);
      }
    }
    return ll;
  }
};

}  // namespace yfm

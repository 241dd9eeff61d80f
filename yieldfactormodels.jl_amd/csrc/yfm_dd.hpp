// yfm_dd.hpp — double-double ("dd", ~106-bit significand) arithmetic on the FP64 VALU,
// for the certified TVλ path (yfm_tvl_dd.hip).
//
// Why it exists: a sizeable share of TVλ EKF candidates amplify any FP64 rounding by
// 1e10..1e13 over T = 600 steps (the reference's dZ1 Jacobian makes the filter locally
// expanding), so every FP64 implementation of filter.jl:12-80 — the reference's own dense
// path included — lands up to 1e-4 away from the exact-arithmetic value, and two such
// implementations disagree by as much.  Carrying the recursion in dd makes the kernel's
// local error ~1e-32 instead of ~1e-16, so its result sits orders of magnitude closer to
// exact arithmetic than any FP64 evaluation.
//
// Algorithms: error-free transformations (Knuth TwoSum, Dekker FastTwoSum, FMA TwoProd)
// and the double-word operations of Joldes, Muller & Popescu (ACM TOMS 2017):
// DWTimesDW (relative error ≤ 5u²), DWPlusFP, and a "sloppy" DW+DW whose ABSOLUTE error is
// ≤ ~3u²(|x|+|y|) — the bound the filter needs (an accumulation error small against the
// operands, like exact-arithmetic summation up to 2^-104).
#pragma once
#include <hip/hip_runtime.h>

// Floating-point contraction must stay off in every translation unit that includes this
// header (a fused a·b + c inside TwoSum / TwoProd would break the error-free
// transformations); the pragma below covers the rest of the including file.
#pragma clang fp contract(off)

namespace yfm {

struct dd {
  double hi, lo;
};

__host__ __device__ __forceinline__ dd dd_make(double x) { return {x, 0.0}; }

// s + e = a + b exactly (any magnitudes)
__host__ __device__ __forceinline__ dd two_sum(double a, double b) {
  const double s = a + b;
  const double bb = s - a;
  const double e = (a - (s - bb)) + (b - bb);
  return {s, e};
}
// s + e = a + b exactly, requires |a| ≥ |b| (or a = 0)
__host__ __device__ __forceinline__ dd fast_two_sum(double a, double b) {
  const double s = a + b;
  return {s, b - (s - a)};
}
// p + e = a·b exactly
__host__ __device__ __forceinline__ dd two_prod(double a, double b) {
  const double p = a * b;
  return {p, __builtin_fma(a, b, -p)};
}

__host__ __device__ __forceinline__ dd dd_neg(dd x) { return {-x.hi, -x.lo}; }

// x + y, absolute error ≤ ~3u²(|x| + |y|)
__host__ __device__ __forceinline__ dd dd_add(dd x, dd y) {
  dd s = two_sum(x.hi, y.hi);
  s.lo += x.lo + y.lo;
  return fast_two_sum(s.hi, s.lo);
}
__host__ __device__ __forceinline__ dd dd_sub(dd x, dd y) { return dd_add(x, dd_neg(y)); }
// x + d (d a double)
__host__ __device__ __forceinline__ dd dd_add_d(dd x, double d) {
  dd s = two_sum(x.hi, d);
  s.lo += x.lo;
  return fast_two_sum(s.hi, s.lo);
}
// x·y, relative error ≤ 5u²
__host__ __device__ __forceinline__ dd dd_mul(dd x, dd y) {
  dd p = two_prod(x.hi, y.hi);
  p.lo = __builtin_fma(x.hi, y.lo, __builtin_fma(x.lo, y.hi, p.lo));
  return fast_two_sum(p.hi, p.lo);
}
// x·y left unnormalised (|lo| ≤ ~3u|hi|): for products that only feed sums and products,
// whose error-free steps do not need a normalised operand
__host__ __device__ __forceinline__ dd dd_mul_nn(dd x, dd y) {
  dd p = two_prod(x.hi, y.hi);
  p.lo = __builtin_fma(x.hi, y.lo, __builtin_fma(x.lo, y.hi, p.lo));
  return p;
}
// x·d
__host__ __device__ __forceinline__ dd dd_mul_d(dd x, double d) {
  dd p = two_prod(x.hi, d);
  p.lo = __builtin_fma(x.lo, d, p.lo);
  return fast_two_sum(p.hi, p.lo);
}
// exact scaling by a power of two
__host__ __device__ __forceinline__ dd dd_ldexp(dd x, int k) { return {__builtin_ldexp(x.hi, k), __builtin_ldexp(x.lo, k)}; }
// 1 / y: FP64 seed + one Newton step in dd (relative error ~ u²)
__host__ __device__ __forceinline__ dd dd_rcp(dd y) {
  const double r0 = 1.0 / y.hi;
  const dd e = dd_add_d(dd_neg(dd_mul_d(y, r0)), 1.0);  // 1 − y·r0
  return dd_add_d(dd_mul_d(e, r0), r0);                  // r0 + r0·e
}
__host__ __device__ __forceinline__ dd dd_div(dd x, dd y) { return dd_mul(x, dd_rcp(y)); }
__host__ __device__ __forceinline__ double dd_to_double(dd x) { return x.hi + x.lo; }

// Accumulator with deferred normalisation: Σ terms kept as an exact leading sum (TwoSum) and
// a plain FP64 sum of all trailing parts.  Same accuracy class as repeated dd_add for the
// sums here (≤ a few hundred terms), at 8 ops per dd term instead of 11.
struct dd_acc {
  double hi = 0.0, lo = 0.0;
  __host__ __device__ __forceinline__ void add(dd x) {
    const dd s = two_sum(hi, x.hi);
    hi = s.hi;
    lo += s.lo + x.lo;
  }
  // += a·b without normalising the product
  __host__ __device__ __forceinline__ void add_prod(dd a, dd b) {
    dd p = two_prod(a.hi, b.hi);
    p.lo = __builtin_fma(a.hi, b.lo, __builtin_fma(a.lo, b.hi, p.lo));
    add(p);
  }
  // += a·d (d a double)
  __host__ __device__ __forceinline__ void add_prod_d(dd a, double d) {
    dd p = two_prod(a.hi, d);
    p.lo = __builtin_fma(a.lo, d, p.lo);
    add(p);
  }
  __host__ __device__ __forceinline__ dd value() const { return two_sum(hi, lo); }  // |lo| may exceed |hi| after cancellation

  // σ-split accumulation (Rump, Ogita & Oishi's ExtractScalar): with σ a power of two ≥ n·max|x.hi|
  // over the n terms this accumulator will receive, q = (σ + x.hi) − σ is x.hi rounded to a multiple
  // of ulp(σ) and x.hi − q is exact; every partial sum of the q's is a multiple of ulp(σ) below 2σ, so
  // `hi` stays exact with one plain addition instead of a TwoSum.  The absolute error, ≈ n²·ulp(σ)·u,
  // is in the same class as add()'s (the sums here have ≤ a few hundred terms).
  __host__ __device__ __forceinline__ void add_sx(dd x, double sg) {
    const double q = (sg + x.hi) - sg;
    hi += q;
    lo += (x.hi - q) + x.lo;
  }
  // += a·b: q = fl(σ + a.hi·b.hi) − σ (one FMA: the exact product rounded to a multiple of ulp(σ)),
  // a.hi·b.hi − q to one rounding (|·| ≤ ulp(σ)), plus the cross terms
  __host__ __device__ __forceinline__ void add_prod_sx(dd a, dd b, double sg) {
    const double q = __builtin_fma(a.hi, b.hi, sg) - sg;
    hi += q;
    lo += __builtin_fma(a.hi, b.hi, -q);
    lo = __builtin_fma(a.hi, b.lo, lo);
    lo = __builtin_fma(a.lo, b.hi, lo);
  }
  // += a·d (d a double)
  __host__ __device__ __forceinline__ void add_prod_d_sx(dd a, double d, double sg) {
    const double q = __builtin_fma(a.hi, d, sg) - sg;
    hi += q;
    lo += __builtin_fma(a.hi, d, -q);
    lo = __builtin_fma(a.lo, d, lo);
  }
};

// the split constant for add_sx & co.: a power of two ≥ x (x = terms × bound on |term|); 1 for
// x = 0 and 2^1000 for a non-finite bound (the split then degrades to FP64 accumulation into lo)
__host__ __device__ __forceinline__ double split_const(double x) {
  if (!(x <= 0x1p1000)) return 0x1p1000;
  return __builtin_ldexp(1.0, __builtin_amdgcn_frexp_exp(x));
}

// exp of a dd argument: x = (4096·m + 64·j1 + j2)·ln2/4096 + r, |r| ≤ ln2/8192, e^x = 2^m · 2^(j1/64) · 2^(j2/4096)
// · e^r with both powers of two from a 128-entry dd table (yfm_exp_table.inc, correctly rounded) and e^r − 1 from a
// degree-7 Taylor polynomial (its degree-4..7 tail in FP64: those terms are below 2^-54 of the result) — ≈ 125
// operations instead of the ≈ 320 of the reduction to |r| ≤ ln2/1024 followed by nine squarings it replaced (round 6;
// `tools/dd_exp_check.cpp` measures both against binary128 on 10⁶ arguments).  Relative error ≲ 4u² for |x| ≲ 40, and
// the reduction's k·(ln2/4096)_lo rounding (absolute in r) up to ≈ 2⁻⁹⁸ at |x| ≈ 700 — the class of the old one.
// Arguments beyond the FP64 range give 0 / Inf like exp(); NaN propagates.
static __constant__ double kDdExpTab[128][2] = {
#include "yfm_exp_table.inc"
};
__host__ __device__ __forceinline__ dd dd_exp_core(dd x, const double (*tab)[2]) {
  constexpr double kInvC = 5909.2788874811944;          // 4096/ln 2
  constexpr double kCHi = 0.0001692253858788929;        // nearest double to ln2/4096
  constexpr double kCLo = 5.661735385366942e-21;        // ln2/4096 − kCHi
  if (!(x.hi > -745.2)) return {x.hi != x.hi ? x.hi : 0.0, 0.0};
  if (x.hi > 709.8) return {__builtin_inf(), 0.0};
  const double k = __builtin_rint(x.hi * kInvC);
  const int ki = (int)k;
  const int m = ki >> 12;                    // floor(k / 4096)
  const int j1 = (ki >> 6) & 63, j2 = ki & 63;
  dd r = dd_sub(x, two_prod(k, kCHi));       // k·C_hi exactly
  r = dd_add_d(r, -k * kCLo);
  // e^r − 1 = r·q1, q1 = 1 + r/2 + r²/6 + r³·(1/24 + r/120 + r²/720 + r³/5040)
  const double q4 = __builtin_fma(r.hi, __builtin_fma(r.hi, __builtin_fma(r.hi, 1.9841269841269841e-4, 1.3888888888888889e-3),
                                                      8.3333333333333332e-3), 4.1666666666666664e-2);
  const dd q3 = dd_add(dd{0.16666666666666666, 9.25185853854297e-18}, dd_mul_d(r, q4));
  const dd q2 = dd_add_d(dd_mul(r, q3), 0.5);
  const dd q1 = dd_add_d(dd_mul(r, q2), 1.0);
  const dd s = dd_mul(r, q1);
  const dd t = dd_mul(dd{tab[j1][0], tab[j1][1]}, dd{tab[64 + j2][0], tab[64 + j2][1]});
  const dd e = dd_add(t, dd_mul(t, s));
  return dd_ldexp(e, m);
}
__device__ __forceinline__ dd dd_exp(dd x) { return dd_exp_core(x, kDdExpTab); }

// x^n, n ≥ 0, by binary powering: ⌈log2 n⌉ squarings and popcount(n) products, relative error ≲ (2 log2 n + 2)·4u²
// on top of n times x's own (the TVλ dd filter's e^{−λkΔ} = (e^{−λΔ})^k on integer maturity grids)
__host__ __device__ __forceinline__ dd dd_powi(dd x, int n) {
  dd r = dd_make(1.0);
  while (n > 0) {  // data-dependent trip count (≤ 9 for n < 512)
    if (n & 1) r = dd_mul(r, x);
    n >>= 1;
    if (n) x = dd_mul(x, x);
  }
  return r;
}

// ---- shared by the double-double filters (yfm_tvl_dd.hip, yfm_fixedz_dd.hip) ----

// −λ·m in dd for exp(−λm); a product that overflows (λ near the FP64 range) is −Inf, whose exp is
// 0 as in the reference — TwoProd's error term would be Inf − Inf = NaN there
__host__ __device__ __forceinline__ dd neg_rate(dd lam, double m) {
  const dd p = dd_mul_d(lam, m);
  return __builtin_isfinite(p.hi) ? dd_neg(p) : dd{-(lam.hi * m), 0.0};
}

// Gaussian elimination with partial pivoting (first max |hi|, the getf2 rule) on an n×n dd
// system with R right-hand sides; false on an exact zero pivot (where getrf reports info > 0).
template <int n, int R>
__host__ __device__ __forceinline__ bool dd_gauss(dd (&A)[n][n], dd (&X)[n][R], dd* det_out = nullptr) {
  bool ok = true;
  double sgn = 1.0;
  dd det = dd_make(1.0);
#pragma unroll
  for (int k = 0; k < n; ++k) {
    int p = k;
    double amax = fabs(A[k][k].hi);
#pragma unroll
    for (int i = k + 1; i < n; ++i) {
      const double a = fabs(A[i][k].hi);
      const bool gt = a > amax;
      amax = gt ? a : amax;
      p = gt ? i : p;
    }
    sgn = (p != k) ? -sgn : sgn;
#pragma unroll
    for (int i = k + 1; i < n; ++i) {
      const bool s = (p == i);
#pragma unroll
      for (int c = k; c < n; ++c) {
        const dd a = A[k][c], b = A[i][c];
        A[k][c] = s ? b : a;
        A[i][c] = s ? a : b;
      }
#pragma unroll
      for (int c = 0; c < R; ++c) {
        const dd a = X[k][c], b = X[i][c];
        X[k][c] = s ? b : a;
        X[i][c] = s ? a : b;
      }
    }
    const dd piv = A[k][k];
    ok = ok && (piv.hi != 0.0);
    if (det_out) det = dd_mul(det, piv);
    const dd r = dd_rcp(piv);
#pragma unroll
    for (int i = k + 1; i < n; ++i) {
      const dd l = dd_mul(A[i][k], r);
#pragma unroll
      for (int c = k + 1; c < n; ++c) A[i][c] = dd_sub(A[i][c], dd_mul(l, A[k][c]));
#pragma unroll
      for (int c = 0; c < R; ++c) X[i][c] = dd_sub(X[i][c], dd_mul(l, X[k][c]));
    }
    A[k][k] = r;  // keep the reciprocal pivot for the back substitution
  }
#pragma unroll
  for (int k = n - 1; k >= 0; --k) {
#pragma unroll
    for (int c = 0; c < R; ++c) {
      dd s = X[k][c];
#pragma unroll
      for (int j = k + 1; j < n; ++j) s = dd_sub(s, dd_mul(A[k][j], X[j][c]));
      X[k][c] = dd_mul(s, A[k][k]);
    }
  }
  if (det_out) *det_out = sgn < 0 ? dd_neg(det) : det;
  return ok;
}

// log of a positive dd to ~u² absolute: FP64 seed + one Newton step on e^y = x
__host__ __device__ __forceinline__ dd dd_log(dd x) {
  const double y0 = log(x.hi);
  const dd e = dd_exp(dd_make(-y0));
  const dd t = dd_add_d(dd_mul(x, e), -1.0);  // x·e^{−y0} − 1
  return dd_add_d(t, y0);
}

// transformations.jl:21-26 as written (2y/(1+y) − 1), in dd
__host__ __device__ __forceinline__ dd dd_from_R_to_11(double x) {
  const dd y = dd_exp(dd_make(x));
  if (!(y.hi < __builtin_inf())) return {__builtin_nan(""), 0.0};  // Inf/Inf
  return dd_add_d(dd_div(dd_mul_d(y, 2.0), dd_add_d(y, 1.0)), -1.0);
}

// Sum of an unnormalised dd over the aligned group of L lanes: each butterfly level pairs
// every lane with its partner and both form the same exact-leading-part sum, so all lanes
// of the group end with bitwise the same value.  The pair needs no canonical order: FP addition
// is commutative and TwoSum's error term is the exact a + b − fl(a + b) whichever operand comes
// first, so (own, partner) and (partner, own) give the same bits (round 6: the lane-order selects,
// 8 v_cndmask per value and level, are gone; logliks bitwise unchanged).
template <int LVL>
__host__ __device__ __forceinline__ void pair_exchange(double x, double& a, double& b) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  if constexpr (LVL <= 3) {
    constexpr int ctrl = LVL == 0 ? 0xB1 : LVL == 1 ? 0x4E : LVL == 2 ? 0x141 : 0x140;
    const int plo = __builtin_amdgcn_mov_dpp(lo, ctrl, 0xf, 0xf, true);
    const int phi = __builtin_amdgcn_mov_dpp(hi, ctrl, 0xf, 0xf, true);
    a = x;
    b = __hiloint2double(phi, plo);
  } else if constexpr (LVL == 4) {
    const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    a = __hiloint2double(rh[0], rl[0]);
    b = __hiloint2double(rh[1], rl[1]);
  } else {
    const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    a = __hiloint2double(rh[0], rl[0]);
    b = __hiloint2double(rh[1], rl[1]);
  }
}

// ---- quad exchanges for the lane-distributed 4×4 update (role c = lane & 3 inside each quad) ----
template <int CTRL>
__host__ __device__ __forceinline__ double quad_dpp(double x) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), CTRL, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
// the value held by role S of this lane's quad
template <int S>
__host__ __device__ __forceinline__ dd quad_bcast(dd x) {
  constexpr int ctrl = S | (S << 2) | (S << 4) | (S << 6);
  return {quad_dpp<ctrl>(x.hi), quad_dpp<ctrl>(x.lo)};
}
// the value held by role c ^ R (R = 1, 2, 3)
template <int R>
__host__ __device__ __forceinline__ dd quad_xor(dd x) {
  constexpr int ctrl = (0 ^ R) | ((1 ^ R) << 2) | ((2 ^ R) << 4) | ((3 ^ R) << 6);
  return {quad_dpp<ctrl>(x.hi), quad_dpp<ctrl>(x.lo)};
}
// v[i] for a lane-dependent i in [0, 4): a two-level mux on the bits of i (a chain of i == k selects is turned
// into a scratch-indexed load by the compiler)
__host__ __device__ __forceinline__ dd sel4(const dd (&v)[4], int i) {
  const bool b0 = (i & 1) != 0, b1 = (i & 2) != 0;
  const dd lo = b0 ? v[1] : v[0];
  const dd hi = b0 ? v[3] : v[2];
  return b1 ? hi : lo;
}

template <int LVL>
__host__ __device__ __forceinline__ void acc_level(double& hi, double& lo) {
  double h0, h1, l0, l1;
  pair_exchange<LVL>(hi, h0, h1);
  pair_exchange<LVL>(lo, l0, l1);
  const dd s = two_sum(h0, h1);
  hi = s.hi;
  lo = (l0 + l1) + s.lo;
}

template <int L>
__host__ __device__ __forceinline__ dd group_sum_acc(dd_acc a) {
  double hi = a.hi, lo = a.lo;
  if constexpr (L >= 2) acc_level<0>(hi, lo);
  if constexpr (L >= 4) acc_level<1>(hi, lo);
  if constexpr (L >= 8) acc_level<2>(hi, lo);
  if constexpr (L >= 16) acc_level<3>(hi, lo);
  if constexpr (L >= 32) acc_level<4>(hi, lo);
  if constexpr (L >= 64) acc_level<5>(hi, lo);
  return two_sum(hi, lo);  // |lo| may exceed |hi| after cancellation
}

// ---- twelve group sums at once for the wide groups (L ≥ 16): recursive halving ----
// Levels 0 and 1 (partners lane ^ 1, lane ^ 2) each keep half of the values a lane still carries — it sends the other
// half to its partner, which keeps that half — so levels 2.. add 3 values instead of 12; the sums then travel back
// (the same two partners, no additions).  Every value is summed over the same pairs in the same tree as
// group_sum_acc's butterfly (after two levels the four lanes of a quad hold one quarter each; the later levels pair
// lanes with equal lane & 3, as the butterfly's mirror pairs pair equal quad values), so the results are bitwise its.
// Cost at L = 64: ≈ 480 instructions instead of ≈ 860.
__device__ __forceinline__ void pair_sum(double& hi, double& lo, double ph, double pl) {
  const dd s = two_sum(hi, ph);
  hi = s.hi;
  lo = (lo + pl) + s.lo;
}
// the value of lane ^ X within each 16-lane row, X ∈ {4, 8} (DPP row rotations)
template <int X>
__device__ __forceinline__ double row_xor(double x, bool upper) {
  if constexpr (X == 8) {
    return quad_dpp<0x128>(x);  // row_ror:8
  } else {
    const double a = quad_dpp<0x124>(x);  // row_ror:4  (lane − 4: right for lanes with bit 2 set)
    const double b = quad_dpp<0x12C>(x);  // row_ror:12 (lane + 4)
    return upper ? a : b;
  }
}
template <int L>
__device__ __forceinline__ void group_sum12(const dd_acc (&in)[12], dd (&out)[12]) {
  static_assert(L >= 16 && L <= 64, "wide groups only");
  const int lane = __lane_id();
  const bool b0 = (lane & 1) != 0, b1 = (lane & 2) != 0, b2 = (lane & 4) != 0;
  // level 0: keep values 6·b0 .. 6·b0 + 5
  double h6[6], l6[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const double sh = b0 ? in[k].hi : in[6 + k].hi, sl = b0 ? in[k].lo : in[6 + k].lo;
    h6[k] = b0 ? in[6 + k].hi : in[k].hi;
    l6[k] = b0 ? in[6 + k].lo : in[k].lo;
    pair_sum(h6[k], l6[k], quad_dpp<0xB1>(sh), quad_dpp<0xB1>(sl));
  }
  // level 1: keep values 3·b1 .. 3·b1 + 2 of those six
  double h3[3], l3[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double sh = b1 ? h6[k] : h6[3 + k], sl = b1 ? l6[k] : l6[3 + k];
    h3[k] = b1 ? h6[3 + k] : h6[k];
    l3[k] = b1 ? l6[3 + k] : l6[k];
    pair_sum(h3[k], l3[k], quad_dpp<0x4E>(sh), quad_dpp<0x4E>(sl));
  }
  // levels 2.. over the lanes with the same lane & 3
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    pair_sum(h3[k], l3[k], row_xor<4>(h3[k], b2), row_xor<4>(l3[k], b2));
    pair_sum(h3[k], l3[k], row_xor<8>(h3[k], false), row_xor<8>(l3[k], false));
    if constexpr (L >= 32) {
      double a, b, c, d;
      pair_exchange<4>(h3[k], a, b);
      pair_exchange<4>(l3[k], c, d);
      const dd s = two_sum(a, b);
      h3[k] = s.hi;
      l3[k] = (c + d) + s.lo;
    }
    if constexpr (L >= 64) {
      double a, b, c, d;
      pair_exchange<5>(h3[k], a, b);
      pair_exchange<5>(l3[k], c, d);
      const dd s = two_sum(a, b);
      h3[k] = s.hi;
      l3[k] = (c + d) + s.lo;
    }
    const dd v = two_sum(h3[k], l3[k]);  // group_sum_acc's final normalisation
    h3[k] = v.hi;
    l3[k] = v.lo;
  }
  // back: the partner of level 1 holds the other three of the six, the partner of level 0 the other six
  double g6h[6], g6l[6];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double rh = quad_dpp<0x4E>(h3[k]), rl = quad_dpp<0x4E>(l3[k]);
    g6h[k] = b1 ? rh : h3[k];
    g6l[k] = b1 ? rl : l3[k];
    g6h[3 + k] = b1 ? h3[k] : rh;
    g6l[3 + k] = b1 ? l3[k] : rl;
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const double rh = quad_dpp<0xB1>(g6h[k]), rl = quad_dpp<0xB1>(g6l[k]);
    out[k] = b0 ? dd{rh, rl} : dd{g6h[k], g6l[k]};
    out[6 + k] = b0 ? dd{g6h[k], g6l[k]} : dd{rh, rl};
  }
}

}  // namespace yfm

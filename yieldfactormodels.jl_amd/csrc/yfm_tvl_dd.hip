// yfm_tvl_dd.hip — the TVλ extended-Kalman-filter log-likelihood carried in double-double
// arithmetic (the default precision mode, YFM_PREC_CERTIFIED of include/yfm.h).
//
// Restates, per candidate θ_b, exactly what yfm_tvl.hip does —
//   get_loss                 src/models/kalman/filter.jl:182-209
//   filter! (TVλ EKF)        src/models/kalman/filter.jl:12-80 (dZ1 = z/λ − z/(λ²m), :43)
//   update_factor_loadings!  src/models/kalman/tvλdns.jl:53-64
//   initialize_filter        src/models/kalman/filter.jl:1-10
//   transform / set_params!  parameteroperations.jl:22-32, paramoperations.jl:6-68
// — but with every quantity that feeds the state recursion (θ_c, λ, the loadings, the
// innovation, the 14 sufficient statistics, the 4×4 capacitance solve, β and P) held as an
// unevaluated sum of two doubles (yfm_dd.hpp).  Why: for a share of candidates the EKF's
// own dynamics amplify a rounding by 1e10..1e13 over T = 600 steps, so any FP64 evaluation,
// the reference's included, is up to 1e-4 from the exact value; a dd evaluation is ~1e-20
// from it (measured against the binary128 truth, oracle/yfm_truth.c).
// The loglik terms themselves (log|det B̃|, v'F⁻¹v) are well conditioned and are summed in
// dd from FP64-rounded values.
//
// Mapping as yfm_tvl.hip: one filter per group of L lanes, lane j owning maturities
// i ≡ j (mod L); per step each lane forms its share of the loadings and statistics, the
// group reduces them with DPP / permlane butterflies (dd-exact pairwise sums), and every
// lane of the group runs the 4×4 update.  Decoding and initialize_filter run in dd in
// tvl_dd_init_kernel (one thread per candidate) and hand over a per-candidate record.
// exp(−λ m_i) walks the maturities of a lane with the dd jump factors e^{−λ d_k}
// (relative drift ≤ (N/L)·2^-104).
#include "yfm_dd.hpp"
#include "yfm_device.hpp"
#include "yfm_internal.hpp"

// Variants measured and not kept (in git history): the statistics in a moment basis Σ z^a·c_i
// (−7% time, but the Jacobian-column sums cancel: 1.1e-8 from the binary128 truth), two waves per SIMD at L = 8
// under a 256-register cap (24.8 vs 21.8 ms), TwoSum instead of σ-split accumulation of the Jacobian-column sums.

namespace yfm {

namespace {

constexpr int kDdBlock = 256;
constexpr int kDdPre = 8;  // panel doubles prefetched per thread per chunk
constexpr int M4 = 4;
// per-group jump factors e^{−λ d_k} in LDS: 17 dd (272 B) apart, so the 16 groups of a wave
// reading their own table hit disjoint banks (a power-of-two stride is a 4-way conflict)
constexpr int kDdJumps = kTvlPowGaps > kTvlGaps ? kTvlPowGaps : kTvlGaps;
constexpr int kDdWStride = kDdJumps + 1;
// per-group 4×4 dd exchange blocks 17 dd (272 B) apart: at 16 dd (256 B = 64 banks) the 16 groups of a wave
// exchanging the same entry all hit the same banks — a 16-way conflict on every transpose
constexpr int kXchStride = 4 * 4 + 1;

// per-candidate record written by tvl_dd_init_kernel (doubles)
constexpr int kDSig = 0;     // σ² (dd)
constexpr int kDDelta = 2;   // δ (4 doubles, exact θ entries)
constexpr int kDPhi = 6;     // Φ row-major (16 dd)
constexpr int kDQ = 38;      // Q upper triangle, row-major i ≤ k (10 dd)
constexpr int kDBeta = 58;   // β₀ (4 dd)
constexpr int kDP = 66;      // P₀ upper triangle (10 dd)
constexpr int kDOk = 86;
constexpr int kDRecLen = 88;
constexpr int kDPar = 58;    // σ², δ, Φ, Q: the read-only part staged in LDS per group

__device__ __forceinline__ int utri(int i, int k) { return i * M4 - i * (i - 1) / 2 + (k - i); }  // i ≤ k < 4

// β ← δ + Φ b;  P ← Φ X Φ'·s + Q  (X symmetric, upper triangle; s = σ² after an update, 1 for
// the prediction-only step)
__device__ __forceinline__ void dd_propagate(const double* par, const dd (&b)[M4], const dd (&X)[10], bool scale,
                                             dd (&beta)[M4], dd (&P)[10]) {
  const dd* Phi = reinterpret_cast<const dd*>(par + kDPhi);
  const dd* Q = reinterpret_cast<const dd*>(par + kDQ);
  const dd sig2 = *reinterpret_cast<const dd*>(par + kDSig);
  dd A[M4][M4];
#pragma unroll
  for (int i = 0; i < M4; ++i) {
    dd s = dd_make(par[kDDelta + i]);
#pragma unroll
    for (int j = 0; j < M4; ++j) s = dd_add(s, dd_mul(Phi[i * M4 + j], b[j]));
    beta[i] = s;
#pragma unroll
    for (int j = 0; j < M4; ++j) {
      dd_acc a;
#pragma unroll
      for (int l = 0; l < M4; ++l) a.add_prod(Phi[i * M4 + l], X[l <= j ? utri(l, j) : utri(j, l)]);
      A[i][j] = a.value();
    }
  }
#pragma unroll
  for (int i = 0; i < M4; ++i)
#pragma unroll
    for (int k = i; k < M4; ++k) {
      dd_acc a;
#pragma unroll
      for (int l = 0; l < M4; ++l) a.add_prod(A[i][l], Phi[k * M4 + l]);
      dd s = a.value();
      if (scale) s = dd_mul(s, sig2);
      P[utri(i, k)] = dd_add(s, Q[utri(i, k)]);
    }
}

// x of the lane at byte address `addr` (= lane · 4) of this wave (ds_bpermute: the LDS crossbar, no LDS memory)
__device__ __forceinline__ double lane_read(int addr, double x) {
  const int lo = __builtin_amdgcn_ds_bpermute(addr, __double2loint(x));
  const int hi = __builtin_amdgcn_ds_bpermute(addr, __double2hiint(x));
  return __hiloint2double(hi, lo);
}

// LDS writes of this wave visible to its own later reads (the quads of a filter are in one wave)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// the dd held by lane S of this lane's 16-lane row (DPP row_newbcast)
template <int S>
__device__ __forceinline__ dd row_bcast(dd x) {
  return {quad_dpp<0x150 + S>(x.hi), quad_dpp<0x150 + S>(x.lo)};
}

template <int S>
__device__ __forceinline__ void bcast_row(const dd (&v)[M4], dd (&out)[M4]) {
#pragma unroll
  for (int k = 0; k < M4; ++k) out[k] = quad_bcast<S>(v[k]);
}
// the symmetric 4×4 whose column `qr` each role qr of the quad holds, in every lane
__device__ __forceinline__ void gather_sym(const dd (&col)[M4], dd (&X)[M4][M4]) {
  bcast_row<0>(col, X[0]);
  bcast_row<1>(col, X[1]);
  bcast_row<2>(col, X[2]);
  bcast_row<3>(col, X[3]);
}

// dd_propagate distributed over the quad (role qr = lane & 3; lanes of a group with the same role
// compute the same values): β_qr then a broadcast; column qr of A = ΦX from column qr of X (the entry role i of the
// row form would form, in the same operation order), one gather; then column qr of the new P.  Every upper entry
// (i ≤ k) is formed by role k exactly as dd_propagate forms it, and the entry below the diagonal is taken from the
// role that owns it as an upper entry, so P stays bitwise symmetric and bitwise dd_propagate's.  xc: column qr of
// the symmetric X.
// xch: this filter's 4×4 dd exchange block in LDS (the transpose of the new P's columns).  The transpose by quad DPP
// exchanges instead (no wave barriers) measured slower even at L = 64, where the step is latency-bound (B = 1: 7.30 vs
// 7.15 ms; profiles/r6/tvl_latency/run1): a dd lane-dependent select costs more than the barrier it removes.
// SPLIT (L ≥ 16: four quads per 16-lane row, qg = the quad's index in its row): lane (qr, qg) forms only entry qg
// of column qr of A and entry qg of column qr of the new P — the same operations in the same order as the role's full
// column, so the result is bitwise the unsplit one — and row qg of A comes from its own quad (one quad broadcast per
// entry instead of the 4×4 gather).  A quarter of the propagation's products per lane on the latency-bound wide groups.
template <bool SPLIT>
__device__ __forceinline__ void dd_propagate_q(const double* par, int qr, int qg, const dd (&b)[M4], const dd (&xc)[M4],
                                               bool scale, dd* xch, dd (&beta)[M4], dd (&Pc)[M4]) {
  const dd* Phi = reinterpret_cast<const dd*>(par + kDPhi);
  const dd* Q = reinterpret_cast<const dd*>(par + kDQ);
  const dd sig2 = *reinterpret_cast<const dd*>(par + kDSig);
  {
    dd s = dd_make(par[kDDelta + qr]);
#pragma unroll
    for (int j = 0; j < M4; ++j) s = dd_add(s, dd_mul(Phi[qr * M4 + j], b[j]));
    beta[0] = quad_bcast<0>(s);
    beta[1] = quad_bcast<1>(s);
    beta[2] = quad_bcast<2>(s);
    beta[3] = quad_bcast<3>(s);
  }
  if constexpr (SPLIT) {
    dd ac;
    {
      dd_acc a;
#pragma unroll
      for (int l = 0; l < M4; ++l) a.add_prod(Phi[qg * M4 + l], xc[l]);
      ac = a.value();  // A[qg][qr]
    }
    const dd ar[M4] = {quad_bcast<0>(ac), quad_bcast<1>(ac), quad_bcast<2>(ac), quad_bcast<3>(ac)};  // row qg of A
    dd pc;
    {
      dd_acc a;
#pragma unroll
      for (int l = 0; l < M4; ++l) a.add_prod(ar[l], Phi[qr * M4 + l]);
      dd s = a.value();
      if (scale) s = dd_mul(s, sig2);
      pc = dd_add(s, Q[qg <= qr ? utri(qg, qr) : utri(qr, qg)]);
    }
    xch[qr * M4 + qg] = pc;
    wave_sync();
#pragma unroll
    for (int k = 0; k < M4; ++k) Pc[k] = xch[k <= qr ? qr * M4 + k : k * M4 + qr];
    wave_sync();  // the block is rewritten by the next exchange
    return;
  }
  dd At[M4][M4];  // At[l][i] = A[i][l]
  {
    dd Ac[M4];
#pragma unroll
    for (int i = 0; i < M4; ++i) {
      dd_acc a;
#pragma unroll
      for (int l = 0; l < M4; ++l) a.add_prod(Phi[i * M4 + l], xc[l]);
      Ac[i] = a.value();
    }
    gather_sym(Ac, At);  // role l's column l of A, in every lane
  }
  dd pc[M4];
#pragma unroll
  for (int i = 0; i < M4; ++i) {
    dd_acc a;
#pragma unroll
    for (int l = 0; l < M4; ++l) a.add_prod(At[l][i], Phi[qr * M4 + l]);
    dd s = a.value();
    if (scale) s = dd_mul(s, sig2);
    pc[i] = dd_add(s, Q[i <= qr ? utri(i, qr) : utri(qr, i)]);
  }
  // role qr's value of entry (k, qr) is its own for k ≤ qr and role k's upper entry (qr, k) below
#pragma unroll
  for (int k = 0; k < M4; ++k) xch[qr * M4 + k] = pc[k];
  wave_sync();
#pragma unroll
  for (int k = 0; k < M4; ++k) {
    const dd o = xch[k * M4 + qr];
    Pc[k] = k <= qr ? pc[k] : o;
  }
  wave_sync();  // the block is rewritten by the next exchange
}

}  // namespace

// decode θ_b in dd (transform_params + set_params!) and run initialize_filter (filter.jl:1-10)
__global__ __launch_bounds__(64) void tvl_dd_init_kernel(const double* __restrict__ theta, int P, int B, int space,
                                                         double* __restrict__ rec, unsigned int* __restrict__ flags_next) {
  if (flags_next && blockIdx.x == 0 && threadIdx.x < kFlagsPerBank) flags_next[threadIdx.x] = 0u;  // the next launch's counters
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const double* th = theta + (size_t)b * P;
  double* r = rec + (size_t)b * kDRecLen;
  int k = 0;
  const dd sig2 = space == 0 ? dd_exp(dd_make(th[k])) : dd_make(th[k]);
  ++k;
  dd U[M4][M4];
#pragma unroll
  for (int j = 0; j < M4; ++j)
#pragma unroll
    for (int i = 0; i < M4; ++i) {
      if (i <= j) {
        const double x = th[k++];
        U[i][j] = (i == j && space == 0) ? dd_exp(dd_make(x)) : dd_make(x);
      } else {
        U[i][j] = dd_make(0.0);
      }
    }
  dd Q[M4][M4];
#pragma unroll
  for (int i = 0; i < M4; ++i)
#pragma unroll
    for (int j = 0; j < M4; ++j) {
      dd_acc a;
#pragma unroll
      for (int l = 0; l < M4; ++l) a.add_prod(U[l][i], U[l][j]);  // Q = U'U
      Q[i][j] = a.value();
    }
  double delta[M4];
#pragma unroll
  for (int i = 0; i < M4; ++i) delta[i] = th[k++];
  dd Phi[M4][M4];
#pragma unroll
  for (int i = 0; i < M4; ++i)
#pragma unroll
    for (int j = 0; j < M4; ++j) {
      const double x = th[k++];
      Phi[i][j] = (i == j && space == 0) ? dd_from_R_to_11(x) : dd_make(x);
    }
  // β₀ = (I − Φ) \ δ
  dd A[M4][M4], x[M4][1];
#pragma unroll
  for (int i = 0; i < M4; ++i) {
#pragma unroll
    for (int j = 0; j < M4; ++j) A[i][j] = (i == j) ? dd_add_d(dd_neg(Phi[i][j]), 1.0) : dd_neg(Phi[i][j]);
    x[i][0] = dd_make(delta[i]);
  }
  bool ok = dd_gauss<M4, 1>(A, x);
  // P₀: the 10 unknowns P_ij (i ≤ j) of P − ΦPΦ' = Q (singular iff I − Φ⊗Φ is)
  constexpr int S = 10;
  dd Ls[S][S], qv[S][1];
  int rr = 0;
#pragma unroll
  for (int i = 0; i < M4; ++i)
#pragma unroll
    for (int j = i; j < M4; ++j) {
      int c = 0;
#pragma unroll
      for (int kk = 0; kk < M4; ++kk)
#pragma unroll
        for (int l = kk; l < M4; ++l) {
          dd s = dd_mul(Phi[i][kk], Phi[j][l]);
          if (kk != l) s = dd_add(s, dd_mul(Phi[i][l], Phi[j][kk]));
          Ls[rr][c] = (rr == c) ? dd_add_d(dd_neg(s), 1.0) : dd_neg(s);
          ++c;
        }
      qv[rr][0] = Q[i][j];
      ++rr;
    }
  ok = dd_gauss<S, 1>(Ls, qv) && ok;
  r[kDSig] = sig2.hi;
  r[kDSig + 1] = sig2.lo;
  int q = 0;
#pragma unroll
  for (int i = 0; i < M4; ++i) {
    r[kDDelta + i] = delta[i];
    r[kDBeta + 2 * i] = x[i][0].hi;
    r[kDBeta + 2 * i + 1] = x[i][0].lo;
#pragma unroll
    for (int j = 0; j < M4; ++j) {
      r[kDPhi + 2 * (i * M4 + j)] = Phi[i][j].hi;
      r[kDPhi + 2 * (i * M4 + j) + 1] = Phi[i][j].lo;
    }
#pragma unroll
    for (int j = i; j < M4; ++j, ++q) {
      r[kDQ + 2 * q] = Q[i][j].hi;
      r[kDQ + 2 * q + 1] = Q[i][j].lo;
      r[kDP + 2 * q] = qv[q][0].hi;
      r[kDP + 2 * q + 1] = qv[q][0].lo;
    }
  }
  r[kDOk] = ok ? 1.0 : 0.0;
  r[kDOk + 1] = 0.0;
}

// Σ_i y_it and Σ_i y_it² per panel column in dd (summed in maturity order; NaN columns give
// NaN and are never read): colsum[4t .. 4t+3] = (Σy.hi, Σy.lo, Σy².hi, Σy².lo); colsum[4T + t] =
// max_i |y_it| (the bound of the σ-split statistics' y terms)
__global__ __launch_bounds__(64) void tvl_dd_colsum_kernel(const double* __restrict__ Y, int N, int T,
                                                           double* __restrict__ colsum) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  const double* y = Y + (size_t)t * N;
  dd_acc s1, s2;
  double ym = 0.0;
  for (int i = 0; i < N; ++i) {
    const double v = y[i];
    s1.add(dd_make(v));
    s2.add(two_prod(v, v));
    ym = fmax(ym, fabs(v));
  }
  colsum[4 * (size_t)T + t] = ym;
  const dd a = s1.value(), b = s2.value();
  colsum[4 * (size_t)t] = a.hi;
  colsum[4 * (size_t)t + 1] = a.lo;
  colsum[4 * (size_t)t + 2] = b.hi;
  colsum[4 * (size_t)t + 3] = b.lo;
}

template <int L, bool RECORD, bool LONG = false>
__global__ __launch_bounds__(kDdBlock, 1) void tvl_dd_loglik_kernel(
    const double* __restrict__ rec, int B, const double* __restrict__ Y, const double* __restrict__ colsum,
    const double* __restrict__ prep, int ldp,
    int np, int T, int N, int TC, const double* __restrict__ mats, int K, const double* __restrict__ gap_d,
    const int* __restrict__ gap_idx, double pstep, const int* __restrict__ T_use, double* __restrict__ out,
    unsigned int* __restrict__ flags, double* __restrict__ rec_beta, double* __restrict__ rec_P, int horizon,
    int rec_len) {
  constexpr int GPB = kDdBlock / L;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  constexpr int kSumDd = 2;                            // dd column sums per staged column
  double* s_m = smem;                                  // m_i
  dd* s_rm = reinterpret_cast<dd*>(smem + N);          // 1/m_i (dd)
  double* s_nan = smem + 3 * N;                        // TC NaN flags of the staged chunk
  dd* s_sum = reinterpret_cast<dd*>(s_nan + TC);       // per staged column: Σy, Σy² (dd)
  double* s_ymax = s_nan + (1 + 2 * kSumDd) * TC;      // per staged column: max_i |y_i|
  double* s_y = s_ymax + TC;                           // TC columns of N yields
  double* s_par = s_y + TC * N;                        // per group: σ², δ, Φ, Q (kDPar doubles)
  dd* s_w = reinterpret_cast<dd*>(s_par + GPB * kDPar);  // per group: e^{-λ d_k}, k < K
  dd* s_xch = s_w + GPB * kDdWStride;                  // per group: 4×4 dd exchange block
  int* s_gi = reinterpret_cast<int*>(s_xch + GPB * kXchStride);
  // jump k: the maturity difference d_k, or (power mode, pstep = Δ > 0) its exponent e_k: e^{−λd_k} = (e^{−λΔ})^{e_k}
  __shared__ double s_gd[kDdJumps];
  __shared__ int s_gsrc[kDdJumps];  // a lane whose first maturity equals jump k exactly, or −1
  __shared__ int s_nobs_max;

  const int tid = threadIdx.x;
  const int j = tid % L;
  const int grp = tid / L;
  const int b = blockIdx.x * GPB + grp;
  const bool live = b < B;
  const int bb = live ? b : (B - 1);
  const int nobs = T_use ? T_use[bb] : T;

  if (tid == 0) s_nobs_max = 0;
  for (int i = tid; i < N; i += kDdBlock) {
    const double m = mats[i];
    s_m[i] = m;
    s_rm[i] = dd_rcp(dd_make(m));
    if (K > 0) s_gi[i] = gap_idx[i];
  }
  if (tid < K) {
    const double d = gap_d[tid];
    s_gd[tid] = d;
    int src = -1;
    if (pstep == 0.0)
      for (int q = min(L, N) - 1; q >= 0; --q) src = mats[q] == d ? q : src;
    s_gsrc[tid] = src;
  }
  const double* r = rec + (size_t)bb * kDRecLen;
  double* par = s_par + grp * kDPar;
  for (int q = j; q < kDPar; q += L) par[q] = r[q];
  __syncthreads();
  // this lane's maturities i ≡ j (mod L): count and smallest maturity (bounds of the σ-split sums)
  double l_n = 0.0, l_minm = __builtin_inf(), l_maxm = 0.0;
  for (int i = j; i < N; i += L) {
    l_n += 1.0;
    l_minm = fmin(l_minm, s_m[i]);
    l_maxm = fmax(l_maxm, s_m[i]);
  }
  const double l_rminm = 1.0 / l_minm;
  const int my_steps = horizon > 0 ? nobs + horizon : nobs - 1;
  const int my_data = horizon > 0 ? nobs : nobs - 1;
  atomicMax(&s_nobs_max, live ? my_steps : 0);

  // the 4×4 update is distributed over the lanes of each quad: role qr holds column qr of P
  const int qr = tid & 3;
  constexpr bool SPLIT = L >= 16;  // the 4×4 update's entries spread over the four quads of a 16-lane row
  const int qg = (tid >> 2) & 3;
  constexpr int kUnrollK1 = LONG ? 2 : 1;  // the one-jump maturity loop (below)
  constexpr bool FACT = L <= 8;              // 1/λ factored out of the z2 sums (below)
  dd* xch = s_xch + grp * kXchStride;
  dd beta[M4], Pc[M4];
#pragma unroll
  for (int i = 0; i < M4; ++i) {
    beta[i] = {r[kDBeta + 2 * i], r[kDBeta + 2 * i + 1]};
    const int q = i <= qr ? utri(i, qr) : utri(qr, i);
    Pc[i] = {r[kDP + 2 * q], r[kDP + 2 * q + 1]};
  }
  const bool init_ok = r[kDOk] != 0.0;
  const dd sig2 = {par[kDSig], par[kDSig + 1]};
  const dd rsig2 = dd_rcp(sig2);

  dd_acc sum_ld, sum_q;
  bool neg = false;
  double last_ld = -__builtin_inf(), last_q = 0.0;  // fresh model: F = 0 (logdet −Inf), v = 0
  bool last_neg = false;

  __syncthreads();
  const int nsteps = max(s_nobs_max, 0);
  const int CHY = TC * N;

  double pre[kDdPre];
  double pre_nan = 0.0, pre_sum[2 * kSumDd] = {}, pre_ymax = 0.0;
  auto load_chunk = [&](int c) {
    const size_t base = (size_t)c * CHY;
    const size_t lim = (size_t)T * N;
#pragma unroll
    for (int q = 0; q < kDdPre; ++q) {
      const int e = q * kDdBlock + tid;
      const size_t g = base + e;
      pre[q] = (e < CHY && g < lim) ? Y[g] : 0.0;
    }
    const int tc = c * TC + tid;
    const bool own = tid < TC && tc < T;
    pre_nan = own ? prep[(size_t)tc * ldp + np + 2] : 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) pre_sum[q] = own ? colsum[(size_t)tc * 4 + q] : 0.0;
    pre_ymax = own ? colsum[(size_t)T * 4 + tc] : 0.0;
  };
  auto store_chunk = [&]() {
#pragma unroll
    for (int q = 0; q < kDdPre; ++q) {
      const int e = q * kDdBlock + tid;
      if (e < CHY) s_y[e] = pre[q];
    }
    if (tid < TC) {
      s_nan[tid] = pre_nan;
      s_sum[kSumDd * tid] = {pre_sum[0], pre_sum[1]};
      s_sum[kSumDd * tid + 1] = {pre_sum[2], pre_sum[3]};
      s_ymax[tid] = pre_ymax;
    }
  };
  if (nsteps > 0) {
    load_chunk(0);
    store_chunk();
    __syncthreads();
    load_chunk(1);
  }

  // the staged column's NaN flag is read one step ahead: the branch at the top of a step would otherwise wait on
  // an LDS read every step (at one wave per SIMD the latency is exposed)
  double nan_next = nsteps > 0 ? s_nan[0] : 0.0;
  for (int t = 0; t < nsteps; ++t) {
    const int tt = t % TC;
    const bool act = live && t < my_steps;
    const bool acc = t >= 1;  // Julia t > 1 (filter.jl:194)
    const bool nan_col = nan_next != 0.0 || t >= my_data;
    if (tt + 1 < TC) nan_next = s_nan[tt + 1];  // the next chunk's first flag is read after its store
    if (act && nan_col) {
      // filter.jl:13-29: prediction only; F, F⁻¹, v stale → the loglik re-adds the last term
      dd bf[M4], xc[M4];
#pragma unroll
      for (int i = 0; i < M4; ++i) {
        bf[i] = beta[i];
        xc[i] = Pc[i];
      }
      dd_propagate_q<SPLIT>(par, qr, qg, bf, xc, false, xch, beta, Pc);
      if (acc) {
        sum_ld.add(dd_make(last_ld));
        sum_q.add(dd_make(last_q));
        neg = neg || last_neg;
      }
    } else if (act) {
      // ---- λ and the per-step constants of the loadings (tvλdns.jl:56, filter.jl:38-46) ----
      const dd e4 = dd_exp(beta[3]);
      const dd lam = dd_add_d(e4, 1e-2);
      const dd dl = dd_add_d(lam, -1e-2);
      const dd rl = dd_rcp(lam);
      // λ near the FP64 range: every z of this lane underflows to 0 and the reference's Jacobian column is 0·dλ
      // (yfm_tvl.hip) — the constants become 0·dλ rather than overflowed (Inf, NaN) pairs or a c2·m_max beyond the
      // range (randomized sweep case 4985: λ = 3.6e304, c2 finite)
      const dd c1r = dd_mul(dd_add(beta[1], beta[2]), dl), c2r = dd_mul(beta[2], dl);
      const bool big = !(lam.hi * l_minm <= 746.0) || !(fabs(c1r.hi) <= __DBL_MAX__) || !(fabs(c2r.hi) <= __DBL_MAX__);
      const dd c1 = big ? dd_make(0.0 * dl.hi) : c1r;
      const dd c2 = big ? dd_make(0.0 * dl.hi) : c2r;
      const dd k1 = dd_mul(c1, rl);
      const double* col = s_y + tt * N;
      const dd kr = dd_mul(k1, rl);
      // Per maturity only the loadings and their products with each other and with y, in the
      // basis (z2, z, z4) — z3 = z2 − z is recovered per step below.  The innovation sums are
      // recovered per step too: u = Z'y − Z'Z[:,1:3]β[1:3] and v'v = y'y − y'ŷ − ŷ'v, which in
      // dd keeps ≥ 80 of 106 bits where the FP64 kernel (yfm_tvl.hip) forms v per maturity.
      // FACT (L ≤ 8): z2 = (1 − z)/(λm) = w2/λ with w2 = (1 − z)/m — the lanes accumulate w2 and its products and
      // the group sums are scaled by 1/λ (1/λ² for Σ w2²) once per step, one dd product per maturity fewer (config 3
      // 19.06 → 17.76 ms); at L = 64 (six maturities per lane, the step latency-bound) it measured 5% slower
      // (profiles/r6/tvl_latency/c24/), so the wide groups keep z2 per maturity.
      // The sums of z, z2 (w2) and their products with each other and with y are σ-split accumulations
      // (yfm_dd.hpp: dd_acc::add_sx): per step and lane, a tight bound on the terms over this lane's
      // maturities (z = e^{−λm} ≤ e^{−λ m_min}, z2 = (1 − z)/(λm) ≤ min(1, 1/(λ m_min)), w2 ≤ min(1/m_min, λ),
      // |y| ≤ the column's max) fixes the split constant.
      const double lamh = lam.hi, rlh = rl.hi;
      constexpr double kSlack = 1.0 + 0x1p-30;
      const double Be = exp(-(lamh * l_minm)) * kSlack;
      const double Bz2 = (FACT ? fmin(l_rminm, lamh) : fmin(1.0, rlh * l_rminm)) * kSlack;
      const double By = s_ymax[tt] * l_n;
      // t = k1 − kr/m + c2·m per maturity, σ-split with the bound of its three terms (k1's split once per step)
      const double sgt = split_const((fabs(k1.hi) + fabs(kr.hi) * l_rminm + fabs(c2.hi) * l_maxm) * kSlack);
      const double qk1 = (sgt + k1.hi) - sgt;
      const double rk1 = (k1.hi - qk1) + k1.lo;
      const double Bem = (lamh * l_minm >= 1.0 ? Be * l_minm : 0.36787944117144233 * rlh) * kSlack;
      const double B4 = (Be * (fabs(k1.hi) + fabs(kr.hi) * l_rminm) + fabs(c2.hi) * Bem) * kSlack;
      const double sg4 = split_const(l_n * B4), sg24 = split_const(l_n * Bz2 * B4);
      const double sgz4 = split_const(l_n * Be * B4), sg44 = split_const(l_n * B4 * B4);
      const double sy4 = split_const(By * B4);
      const double sg2 = split_const(l_n * Bz2), sgz = split_const(l_n * Be);
      const double sg22 = split_const(l_n * Bz2 * Bz2), sg2z = split_const(l_n * Bz2 * Be);
      const double sgzz = split_const(l_n * Be * Be);
      const double sy2 = split_const(By * Bz2), syz = split_const(By * Be);
      dd_acc S2, Sz, S4, G22, G2z, G24, Gzz, Gz4, G44, Y2, Yz, Y4;
      auto accum = [&](double m, double y, dd rm, dd z) {
        // 1 − z exactly (Fast2Sum: 1 ≥ z.hi), then z2 = (1 − z)/τ (FACT: w2 = (1 − z)/m = λ·z2)
        const double o1 = 1.0 - z.hi;
        const dd ome = {o1, ((1.0 - o1) - z.hi) - z.lo};
        const dd z2 = FACT ? dd_mul_nn(ome, rm) : dd_mul_nn(ome, dd_mul_nn(rl, rm));
        // ((β2+β3)(z/λ − z/(λ²m)) + β3·m·z)·(λ − 0.01) = z·t,  t = k1(1 − 1/τ) + c2·m
        // (t left unnormalised: its products are formed to an absolute error of ~2^-104·|terms|)
        dd ta;
        {
          const double q1 = __builtin_fma(-kr.hi, rm.hi, sgt) - sgt;
          const double l1 = __builtin_fma(-kr.hi, rm.lo, __builtin_fma(-kr.lo, rm.hi, __builtin_fma(-kr.hi, rm.hi, -q1)));
          const double q2 = __builtin_fma(c2.hi, m, sgt) - sgt;
          const double l2 = __builtin_fma(c2.lo, m, __builtin_fma(c2.hi, m, -q2));
          ta.hi = (qk1 + q1) + q2;  // exact: multiples of ulp(σ) below σ
          ta.lo = (rk1 + l1) + l2;
        }
        const dd z4 = dd_mul_nn(z, ta);
        S2.add_sx(z2, sg2);
        Sz.add_sx(z, sgz);
        G22.add_prod_sx(z2, z2, sg22);
        G2z.add_prod_sx(z2, z, sg2z);
        Gzz.add_prod_sx(z, z, sgzz);
        Y2.add_prod_d_sx(z2, y, sy2);
        Yz.add_prod_d_sx(z, y, syz);
        S4.add_sx(z4, sg4);
        G24.add_prod_sx(z2, z4, sg24);
        Gz4.add_prod_sx(z, z4, sgz4);
        G44.add_prod_sx(z4, z4, sg44);
        Y4.add_prod_d_sx(z4, y, sy4);
      };
      if (K > 0) {
        dd* w = s_w + grp * kDdWStride;
        dd z;
        // one jump equal to some lane's first maturity (uniform grids): the factor is that lane's start value,
        // read across the group with ds_bpermute — no LDS block, no wave barrier on the step's serial path
        const bool jump1 = pstep == 0.0 && K == 1 && s_gsrc[0] >= 0;  // block-uniform
        if (pstep > 0.0) {
          // power mode: one dd exp, b = e^{−λΔ}; the lane's start value and the group's jump factors are integer
          // powers of it (m_j/Δ and e_q are exact integers) — in place of one dd exp per maturity
          // The squarings b^(2^k) are formed once per step and shared by the lane's powers (dd_powi squares again in
          // every call): each power is then the same products of the same factors in the same order — bitwise
          // dd_powi's — at one dd product per set bit (jump exponents < 512: the host's power table)
          const dd bs = dd_exp(neg_rate(lam, pstep));
          dd sq[9];
          sq[0] = bs;
#pragma unroll
          for (int k = 1; k < 9; ++k) sq[k] = dd_mul(sq[k - 1], sq[k - 1]);
          auto pow_sq = [&](int n) {
            dd r = dd_make(1.0);
#pragma unroll
            for (int k = 0; k < 9; ++k)
              if ((n >> k) & 1) r = dd_mul(r, sq[k]);
            return r;
          };
          const int n0 = (int)(s_m[j] / pstep);
          z = (j < N) ? (n0 < 512 ? pow_sq(n0) : dd_powi(bs, n0)) : dd_make(0.0);
          for (int q = j; q < K; q += L) w[q] = pow_sq((int)s_gd[q]);
        } else {
          z = (j < N) ? dd_exp(neg_rate(lam, s_m[j])) : dd_make(0.0);
          // a jump equal to some lane's first maturity (uniform grids: d = L·Δ = m_{L−1}) is that
          // lane's start value — the same dd_exp of the same argument — so only the others cost an exp
          if (!jump1) {
            for (int q = 0; q < K; ++q)
              if (s_gsrc[q] == j) w[q] = z;
            for (int q = j; q < K; q += L)
              if (s_gsrc[q] < 0) w[q] = dd_exp(neg_rate(lam, s_gd[q]));
          }
        }
        if (!jump1) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        // the LDS operands of maturity i + L are read while maturity i is accumulated (at one wave per SIMD a
        // read at the top of the iteration it feeds stalls the wave for the LDS latency); the last read is a
        // harmless repeat of maturity N − 1.  LONG (≥ 32 maturities per lane: config 3's 90 at L = 4): the one-jump
        // loop unrolled by two, the register sets alternating instead of being moved (136 → 126.5 instructions per
        // maturity, 19.3 → 19.0 ms); short loops (L = 64 at N = 360, the estimator's N = 30 rounds) keep the plain
        // instantiation — the unrolled one measured 2–4% slower there (profiles/r6/tvl_latency/c20/, c20b/)
        const int last = N - 1;
        const int i0 = min(j, last);
        double m_n = s_m[i0], y_n = col[i0];
        dd rm_n = s_rm[i0];
        if (K == 1) {
          // one jump (uniform grids): the factor is loop-invariant
          dd wn;
          if (jump1) {
            const int src = ((tid & 63) - j + s_gsrc[0]) << 2;  // the source lane of this group (groups are wave-aligned)
            wn = {lane_read(src, z.hi), lane_read(src, z.lo)};
          } else {
            wn = w[0];
          }
#pragma unroll kUnrollK1
          for (int i = j; i < N; i += L) {
            const double m = m_n, y = y_n;
            const dd rm = rm_n;
            const int in = min(i + L, last);
            m_n = s_m[in];
            y_n = col[in];
            rm_n = s_rm[in];
            accum(m, y, rm, z);
            z = FACT ? dd_mul_nn(z, wn) : dd_mul(z, wn);  // FACT: left unnormalised (z only feeds products, σ-split sums and 1 − z)
          }
        } else {
          dd wn_n = w[s_gi[i0]];
          for (int i = j; i < N; i += L) {
            const double m = m_n, y = y_n;
            const dd rm = rm_n, wn = wn_n;
            const int in = min(i + L, last);
            m_n = s_m[in];
            y_n = col[in];
            rm_n = s_rm[in];
            wn_n = w[s_gi[in]];
            accum(m, y, rm, z);
            z = FACT ? dd_mul_nn(z, wn) : dd_mul(z, wn);  // FACT: left unnormalised (z only feeds products, σ-split sums and 1 − z)
          }
        }
      } else {
        for (int i = j; i < N; i += L) accum(s_m[i], col[i], s_rm[i], dd_exp(neg_rate(lam, s_m[i])));
      }
      dd s2, g22, g2z, g24, y2, sz, s4, gzz, gz4, g44, yz, y4;
      if constexpr (L >= 16) {
        // recursive halving (yfm_dd.hpp group_sum12): bitwise the butterfly's sums at about half its cost
        const dd_acc in[12] = {S2, G22, G2z, G24, Y2, Sz, S4, Gzz, Gz4, G44, Yz, Y4};
        dd o[12];
        group_sum12<L>(in, o);
        s2 = o[0]; g22 = o[1]; g2z = o[2]; g24 = o[3]; y2 = o[4];
        sz = o[5]; s4 = o[6]; gzz = o[7]; gz4 = o[8]; g44 = o[9]; yz = o[10]; y4 = o[11];
      } else {
        s2 = group_sum_acc<L>(S2); g22 = group_sum_acc<L>(G22); g2z = group_sum_acc<L>(G2z);
        g24 = group_sum_acc<L>(G24); y2 = group_sum_acc<L>(Y2);
        sz = group_sum_acc<L>(Sz); s4 = group_sum_acc<L>(S4);
        gzz = group_sum_acc<L>(Gzz); gz4 = group_sum_acc<L>(Gz4); g44 = group_sum_acc<L>(G44);
        yz = group_sum_acc<L>(Yz); y4 = group_sum_acc<L>(Y4);
      }
      if constexpr (FACT) {
        const dd rl2 = dd_mul(rl, rl);
        s2 = dd_mul(s2, rl);
        g22 = dd_mul(g22, rl2);
        g2z = dd_mul(g2z, rl);
        g24 = dd_mul(g24, rl);
        y2 = dd_mul(y2, rl);
      }
      // back to the loading basis (1, z2, z3 = z2 − z, z4)
      const dd g23 = dd_sub(g22, g2z);
      dd G[M4][M4];
      G[0][0] = dd_make((double)N);
      G[0][1] = G[1][0] = s2;
      G[0][2] = G[2][0] = dd_sub(s2, sz);
      G[0][3] = G[3][0] = s4;
      G[1][1] = g22;
      G[1][2] = G[2][1] = g23;
      G[1][3] = G[3][1] = g24;
      G[2][2] = dd_add(dd_sub(g23, g2z), gzz);  // Σ(z2 − z)² = g22 − 2 g2z + gzz
      G[2][3] = G[3][2] = dd_sub(g24, gz4);
      G[3][3] = g44;
      const dd y3 = dd_sub(y2, yz);
      // u_c = Σ_i Z_ic (y_i − ŷ_i), ŷ = β1 + β2 z2 + β3 z3;  v'v = y'y − β'(Z'y)[1:3] − β'u[1:3]
      const dd sy = s_sum[kSumDd * tt], syy = s_sum[kSumDd * tt + 1];
      const dd zy[M4] = {sy, y2, y3, y4};
      // entry qg of a row of 4 dd values held in every lane (a bit mux on the halves: a select of dd values becomes a
      // scratch-indexed load)
      const bool qb0 = (qg & 1) != 0, qb1 = (qg & 2) != 0;
      auto selq4 = [qb0, qb1](dd v0, dd v1, dd v2, dd v3) {
        const double h = qb1 ? (qb0 ? v3.hi : v2.hi) : (qb0 ? v1.hi : v0.hi);
        const double o = qb1 ? (qb0 ? v3.lo : v2.lo) : (qb0 ? v1.lo : v0.lo);
        return dd{h, o};
      };
      dd u[M4];
      if constexpr (SPLIT) {
        // lane (qr, qg) forms u[qg] (the same operations), u[c] is then read from lane 4c of the row
        dd_acc a;
        a.add(selq4(sy, y2, y3, y4));
#pragma unroll
        for (int l = 0; l < 3; ++l) a.add_prod(dd_neg(beta[l]), selq4(G[l][0], G[l][1], G[l][2], G[l][3]));  // G[qg][l]
        const dd uq = a.value();
        u[0] = row_bcast<0>(uq);
        u[1] = row_bcast<4>(uq);
        u[2] = row_bcast<8>(uq);
        u[3] = row_bcast<12>(uq);
      } else {
#pragma unroll
        for (int c = 0; c < M4; ++c) {
          dd_acc a;
          a.add(zy[c]);
#pragma unroll
          for (int l = 0; l < 3; ++l) a.add_prod(dd_neg(beta[l]), G[c][l]);
          u[c] = a.value();
        }
      }
      dd vv;
      {
        dd_acc a;
        a.add(syy);
#pragma unroll
        for (int l = 0; l < 3; ++l) {
          a.add_prod(dd_neg(beta[l]), zy[l]);
          a.add_prod(dd_neg(beta[l]), u[l]);
        }
        vv = a.value();
      }

      // ---- capacitance solve: B̃ = σ²I + P G, W = B̃⁻¹P, distributed over the quad:
      // role qr forms row qr of B̃ (P symmetric: its row qr is the column it holds), every lane
      // factorises the broadcast B̃ and solves for ONE right-hand side, column qr of P ----
      dd A[M4][M4];
      if constexpr (SPLIT) {
        // lane (qr, qg): entry (qr, qg) of B̃ (the unsplit role's Ar[qg], same operations); entry (r, k) is in lane 4k + r
        // of the row
        dd_acc a;
        a.add(qg == qr ? sig2 : dd_make(0.0));
#pragma unroll
        for (int l = 0; l < M4; ++l) a.add_prod(Pc[l], selq4(G[l][0], G[l][1], G[l][2], G[l][3]));
        const dd ar = a.value();
        A[0][0] = row_bcast<0>(ar); A[1][0] = row_bcast<1>(ar); A[2][0] = row_bcast<2>(ar); A[3][0] = row_bcast<3>(ar);
        A[0][1] = row_bcast<4>(ar); A[1][1] = row_bcast<5>(ar); A[2][1] = row_bcast<6>(ar); A[3][1] = row_bcast<7>(ar);
        A[0][2] = row_bcast<8>(ar); A[1][2] = row_bcast<9>(ar); A[2][2] = row_bcast<10>(ar); A[3][2] = row_bcast<11>(ar);
        A[0][3] = row_bcast<12>(ar); A[1][3] = row_bcast<13>(ar); A[2][3] = row_bcast<14>(ar); A[3][3] = row_bcast<15>(ar);
      } else {
        dd Ar[M4];
#pragma unroll
        for (int k = 0; k < M4; ++k) {
          dd_acc a;
          a.add(k == qr ? sig2 : dd_make(0.0));
#pragma unroll
          for (int l = 0; l < M4; ++l) a.add_prod(Pc[l], G[l][k]);
          Ar[k] = a.value();
        }
        gather_sym(Ar, A);
      }
      dd x[M4][1];
#pragma unroll
      for (int i = 0; i < M4; ++i) x[i][0] = Pc[i];
      dd det;
      dd_gauss<M4, 1>(A, x, &det);
      // column qr of the symmetric part of W: (W[k][qr] + W[qr][k])/2 with W[qr][k] from role k (for
      // k = qr the same value twice: exactly W[qr][qr]); dd_add commutes bitwise, so the roles agree
      dd ws[M4];
#pragma unroll
      for (int k = 0; k < M4; ++k) xch[qr * M4 + k] = x[k][0];
      wave_sync();
#pragma unroll
      for (int k = 0; k < M4; ++k) ws[k] = dd_ldexp(dd_add(x[k][0], xch[k * M4 + qr]), -1);
      wave_sync();
      // K v = W u: component qr, then all four
      dd kv[M4];
      {
        dd_acc a;
#pragma unroll
        for (int k = 0; k < M4; ++k) a.add_prod(ws[k], u[k]);
        const dd kq = a.value();
        kv[0] = quad_bcast<0>(kq);
        kv[1] = quad_bcast<1>(kq);
        kv[2] = quad_bcast<2>(kq);
        kv[3] = quad_bcast<3>(kq);
      }
      dd bf[M4];
      dd_acc uk;
#pragma unroll
      for (int i = 0; i < M4; ++i) {
        bf[i] = dd_add(beta[i], kv[i]);
        uk.add_prod(u[i], kv[i]);
      }
      const double q = dd_to_double(dd_mul(dd_sub(vv, uk.value()), rsig2));
      const double dh = dd_to_double(det);
      const bool upd = dh != 0.0;  // inv(F) threw: return without updating (filter.jl:51-56)
      if (upd) {
        dd_propagate_q<SPLIT>(par, qr, qg, bf, ws, true, xch, beta, Pc);
      }
      last_ld = upd ? log(fabs(dh)) : -__builtin_inf();
      last_q = upd ? q : __builtin_nan("");
      last_neg = dh < 0.0;
      if (acc) {
        sum_ld.add(dd_make(last_ld));
        sum_q.add(dd_make(last_q));
        neg = neg || last_neg;
      }
    }
    if constexpr (RECORD) {
      const int slot = t - max(0, my_steps - rec_len);
      dd Pf[M4][M4];
      gather_sym(Pc, Pf);  // every lane of the quad takes part in the exchange
      if (act && j == 0 && slot >= 0) {
        const size_t o = (size_t)b * (size_t)rec_len + slot;
#pragma unroll
        for (int i = 0; i < M4; ++i) rec_beta[o * M4 + i] = dd_to_double(beta[i]);
        if (rec_P) {
#pragma unroll
          for (int c = 0; c < M4; ++c)
#pragma unroll
            for (int i = 0; i < M4; ++i) rec_P[o * M4 * M4 + c * M4 + i] = dd_to_double(Pf[i][c]);
        }
      }
    }
    if (tt == TC - 1) {
      __syncthreads();
      store_chunk();
      __syncthreads();
      nan_next = s_nan[0];
      load_chunk(t / TC + 2);
    }
  }

  if (!live || j != 0) return;
  double ll;
  if (!init_ok) {
    ll = __builtin_nan("");
    atomicAdd(&flags[0], 1u);
  } else {
    const int nterms = max(nobs - 2, 0);
    if (nterms == 0) {
      ll = 0.0;
    } else {
      // per term: (N − 4)·log σ² + N·log 2π (+ log|det B̃_t| + q_t, summed above)
      const dd lsig = dd_log(sig2);
      dd tot = dd_mul_d(dd_add_d(dd_mul_d(lsig, (double)(N - M4)), (double)N * kLog2Pi), (double)nterms);
      tot = dd_add(tot, dd_add(sum_ld.value(), sum_q.value()));
      ll = -0.5 * dd_to_double(tot);
    }
    if (neg || !isfinite(ll)) {
      ll = -__builtin_inf();
      atomicAdd(&flags[1], 1u);
    }
  }
  out[b] = ll;
}

namespace {

template <int L>
hipError_t launch_tvl_dd_l(const LaunchArgs& a, const double* rec_dd, const double* colsum, const TvlGaps& g, int TC) {
  constexpr int GPB = kDdBlock / L;
  const int grid = (a.B + GPB - 1) / GPB;
  constexpr int kSumDd = 2;
  // the kernel's LDS layout: m, 1/m, per staged column NaN flag, dd sums, max|y| and N yields, per group the
  // parameters, jump factors and exchange block, and the jump index per maturity
  const size_t shmem = sizeof(double) * (size_t)(3 * a.N + (2 + 2 * kSumDd) * TC + TC * a.N + GPB * kDPar +
                                                 2 * GPB * kDdWStride + 2 * GPB * kXchStride) +
                       sizeof(int) * a.N;
  if (shmem > 160 * 1024) return hipErrorInvalidValue;  // gfx950: 160 KiB of LDS per workgroup
  auto* k = a.rec_beta ? &tvl_dd_loglik_kernel<L, true> : &tvl_dd_loglik_kernel<L, false>;
  if constexpr (L <= 8) {
    if (!a.rec_beta && a.N >= 32 * L) k = &tvl_dd_loglik_kernel<L, false, true>;  // long maturity loops
  }
  if (shmem > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)shmem);
    if (e != hipSuccess) return e;
  }
  // the exact jump table if there is one, else the power mode if the grid allows it, else one exp per maturity
  const bool pw = g.K == 0 && g.Kp > 0;
  hipLaunchKernelGGL(k, dim3(grid), dim3(kDdBlock), shmem, a.stream, rec_dd, a.B, a.raw, colsum, a.panel, a.ldp,
                     a.np, a.T, a.N, TC, a.mats, pw ? g.Kp : g.K, pw ? g.e : g.d, pw ? g.pidx : g.idx,
                     pw ? g.step : 0.0, a.T_use, a.out, a.flags, a.rec_beta, a.rec_P, a.rec_beta ? a.horizon : 0,
                     a.rec_beta ? a.rec_len : 0);
  return hipGetLastError();
}

}  // namespace

// per-candidate records
size_t tvl_dd_scratch_bytes(int B) { return sizeof(double) * (size_t)kDRecLen * (size_t)(B > 0 ? B : 1); }
// the panel's column statistics: 5 doubles per column (tvl_dd_colsum_kernel)
size_t tvl_dd_colsum_bytes(int T) { return sizeof(double) * 5 * (size_t)(T > 0 ? T : 1); }

hipError_t launch_tvl_dd_colsum(const double* Y, int N, int T, double* colsum, hipStream_t s) {
  hipLaunchKernelGGL(tvl_dd_colsum_kernel, dim3((T + 63) / 64), dim3(64), 0, s, Y, N, T, colsum);
  return hipGetLastError();
}

int tvl_dd_lanes_for(int B, int N, int want, int share) {
  // at least 4 lanes per filter (the 4×4 update is distributed over a lane quad, and the per-group parameter block
  // of 256 / L groups must fit the 64 KiB of dynamic LDS a launch gets by default), at most 64 and the maturity
  // count rounded up
  int capN = 4;
  while (capN < N && capN < 64) capN <<= 1;
  if (want > 0) {
    int L = 4;
    while (L < want && L < 64) L <<= 1;
    return L;
  }
  // The L with the least modelled time.  The kernel needs the whole register file (one wave per SIMD, 1,024 on the
  // chip), so waves run in rounds of 1,024; per filter step a wave issues ≈ ⌈N/L⌉·137 instructions of maturity loop,
  // ≈ 4,250 of 4×4 dd update and per-step constants (replicated on every quad of a group) and ≈ 200 per butterfly
  // level (instruction counts of this build's ISA; L ≥ 16 below).  `share` concurrent launches of this size divide the SIMDs.
  // Measured choices it keeps at N = 360: B = 16,384 → 4, B ≤ 1,024 → 64 (profiles/r5/first/c3_B*_L*.json).  At
  // N = 30 the update dominates: the estimator's 7,680-point rounds (two at once) take L = 4, where the round-5
  // rule ("one wave per SIMD of lanes") gave 16 — four rounds of waves instead of one.
  const double waves_unit = (double)(B > 0 ? B : 1) * (share > 0 ? share : 1) / 64.0;
  int best = 4;
  double best_cost = 0.0;
  for (int L = 4, lg = 2; L <= capN; L <<= 1, ++lg) {
    const double rounds = std::ceil(waves_unit * L / 1024.0);
    // L ≥ 16: the update's products split over the four quads of a row and the sums by recursive halving
    // (group_sum12): ≈ 3,650 + 288 + 60 per level after the second (B = 1 at L = 64: 6.48 → 5.17 ms, L = 16 at
    // B = 4,096: 8.97 → 7.84 ms, profiles/r6/tvl_latency/c29b/)
    const double issue = (double)((N + L - 1) / L) * 137.0 +
                         (L >= 16 ? 3650.0 + 288.0 + 60.0 * (lg - 2) : 4250.0 + 200.0 * lg);
    const double cost = rounds * issue;
    if (L == 4 || cost < best_cost) {
      best = L;
      best_cost = cost;
    }
  }
  return best;
}

hipError_t launch_tvl_dd_init(const LaunchArgs& a, double* rec_dd) {
  hipLaunchKernelGGL(tvl_dd_init_kernel, dim3((a.B + 63) / 64), dim3(64), 0, a.stream, a.theta, a.P, a.B, a.space,
                     rec_dd, a.flags_next);
  return hipGetLastError();
}

hipError_t launch_tvl_dd(const LaunchArgs& a, const double* rec_dd, const double* colsum, const TvlGaps& g_in,
                         int lanes) {
  // the recurrence z_{i+L} = z_i·e^{−λ d} is only as exact as the jumps d: a rounded maturity
  // difference would put an FP64-sized error into every loading, so such grids take one dd exp
  // per maturity
  TvlGaps g = g_in;
  if (!g.exact) g.K = 0;
  int TC = (kDdPre * kDdBlock) / a.N;
  if (TC > 32) TC = 32;
  if (TC < 1) return hipErrorInvalidValue;
  switch (lanes) {
    case 4: return launch_tvl_dd_l<4>(a, rec_dd, colsum, g, TC);
    case 8: return launch_tvl_dd_l<8>(a, rec_dd, colsum, g, TC);
    case 16: return launch_tvl_dd_l<16>(a, rec_dd, colsum, g, TC);
    case 32: return launch_tvl_dd_l<32>(a, rec_dd, colsum, g, TC);
    case 64: return launch_tvl_dd_l<64>(a, rec_dd, colsum, g, TC);
  }
  return hipErrorInvalidValue;
}

}  // namespace yfm

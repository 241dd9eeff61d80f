// yfm_fixedz_dd.hip — the fixed-loading models (DNS, GNS5) in double-double arithmetic for the
// candidates the FP64 kernels defer: ill-conditioned loadings (κ₁(Z'Z) ≥ kCollapsedKappa, fewer
// maturities than states, or a singular Z'Z).
//
// Restates, per deferred candidate, the same reference functions as yfm_kernels.hip —
//   get_loss                 src/models/kalman/filter.jl:182-209
//   filter! (fixed Z)        src/models/kalman/filter.jl:125-179
//   update_factor_loadings!  src/models/kalman/dns.jl:51-65 (GNS5: a second (S, C) pair)
//   initialize_filter        src/models/kalman/filter.jl:1-10
//   transform / set_params!  parameteroperations.jl:22-32, paramoperations.jl:6-59
// — in the capacitance form (B̃ = σ²I + PG, W = B̃⁻¹P, K v = W Z'v, P_{t|t} = σ²W,
// v'F⁻¹v = (v'v − u'Wu)/σ², det F = σ^{2(N−M)} det B̃), with every quantity that feeds
// the recursion (θ_c, the loadings, Z'Z, the innovation per maturity and its sums, the M×M
// solve, β and P) held as an unevaluated pair of doubles (yfm_dd.hpp).
//
// Why: on these lanes the FP64 forms lose digits in proportion to the conditioning of what they
// invert — the collapsed form to κ(Z'Z) (R = σ²(Z'Z)⁻¹ and ĉ = (Z'Z)⁻¹Z'y), the FP64
// capacitance form to κ(B̃) through v'v − u'Wu — so an FP64 evaluation there lands 1e-9 … 1e-8
// from the exact value where the reference's dense N×N path (whose F is small or better
// conditioned for these shapes) is 1e-13 … 1e-10 from it.  In dd the same algebra is ~1e-20
// from exact arithmetic (the binary128 restatement, oracle/yfm_truth.c), so the deferred lanes
// are at least as close to the exact value of filter.jl as the reference itself.
//
// Mapping (as yfm_tvl_dd.hip): one filter per group of L lanes; lane j owns maturities
// i ≡ j (mod L) and their dd loadings; per step each lane forms the innovation of its maturities
// and its share of u = Z'v and v'v, the group reduces them with DPP / permlane butterflies
// (dd-exact pairwise sums, every lane ends with the same bits) and every lane runs the M×M
// update.  Decoding and initialize_filter run in dd in fd_init_record (one lane per deferred
// candidate, at the top of its slot) and hand over a per-candidate record.  Deferred lanes are rare (none in the
// benchmark configurations), so the kernels read the deferral list the FP64 kernel
// built on the device and launch one filter slot per candidate of the batch, the slots past the
// list exiting at once.
#include "yfm_dd.hpp"
#include "yfm_device.hpp"
#include "yfm_internal.hpp"

#include <algorithm>

namespace yfm {

namespace {

constexpr int kFdBlock = 256;
constexpr int kFdPre = 8;  // panel doubles prefetched per thread per chunk

// per-candidate record written by fd_init_record (doubles), parametrised by M
template <int M>
struct FdRec {
  static constexpr int U = M * (M + 1) / 2;  // upper-triangle entries
  static constexpr int Sig = 0;              // σ² (dd)
  static constexpr int Delta = 2;            // δ (M doubles, exact θ entries)
  static constexpr int Phi = Delta + M;      // Φ row-major (M² dd)
  static constexpr int Q = Phi + 2 * M * M;  // Q upper triangle, row-major i ≤ k (dd)
  static constexpr int Par = Q + 2 * U;      // σ², δ, Φ, Q: the read-only part staged in LDS per group
  static constexpr int Beta = Par;           // β₀ (M dd)
  static constexpr int P0 = Beta + 2 * M;    // P₀ upper triangle (dd)
  static constexpr int Ok = P0 + 2 * U;
  static constexpr int Len = Ok + 2;
};

template <int M>
__device__ __forceinline__ constexpr int ut(int i, int k) {  // i ≤ k < M
  return i * M - i * (i - 1) / 2 + (k - i);
}
template <int M>
__device__ __forceinline__ constexpr int us(int i, int k) {  // any order
  return i <= k ? ut<M>(i, k) : ut<M>(k, i);
}

// β ← δ + Φ b;  P ← Φ X Φ'·s + Q  (X symmetric, upper triangle; s = σ² after an update)
template <int M>
__device__ __forceinline__ void fd_propagate(const double* par, const dd (&b)[M], const dd (&X)[FdRec<M>::U],
                                             bool scale, dd (&beta)[M], dd (&P)[FdRec<M>::U]) {
  using R = FdRec<M>;
  const dd* Phi = reinterpret_cast<const dd*>(par + R::Phi);
  const dd* Q = reinterpret_cast<const dd*>(par + R::Q);
  const dd sig2 = *reinterpret_cast<const dd*>(par + R::Sig);
  dd A[M][M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    dd_acc s;
    s.add(dd_make(par[R::Delta + i]));
#pragma unroll
    for (int j = 0; j < M; ++j) s.add_prod(Phi[i * M + j], b[j]);
    beta[i] = s.value();
#pragma unroll
    for (int j = 0; j < M; ++j) {
      dd_acc a;
#pragma unroll
      for (int l = 0; l < M; ++l) a.add_prod(Phi[i * M + l], X[us<M>(l, j)]);
      A[i][j] = a.value();
    }
  }
#pragma unroll
  for (int i = 0; i < M; ++i)
#pragma unroll
    for (int k = i; k < M; ++k) {
      dd_acc a;
#pragma unroll
      for (int l = 0; l < M; ++l) a.add_prod(A[i][l], Phi[k * M + l]);
      dd s = a.value();
      if (scale) s = dd_mul(s, sig2);
      P[ut<M>(i, k)] = dd_add(s, Q[ut<M>(i, k)]);
    }
}

}  // namespace

// decode θ_b in dd (transform_params + set_params!) and run initialize_filter (filter.jl:1-10) into the
// record r of one deferred candidate.  Called by one lane of the candidate's group inside
// fixedz_dd_loglik_kernel (round 4: a separate init kernel cost a ~4.4 µs launch on every config-2 call,
// deferred lanes or not).  DNS inlines it (its 6×6 solve fits beside the filter's registers; a call would make
// the kernel save callee registers to scratch, and a kernel with a private segment costs its dispatch even when
// the deferral list is empty); GNS5 calls it out of line (fd_init_record_call) so that its 15×15 dd solve does
// not shape the filter's registers.
template <int M, int LEAD>
__device__ __forceinline__ void fd_init_record(const double* __restrict__ theta, int P, int space, int b,
                                               double* __restrict__ r) {
  using R = FdRec<M>;
  {
  const double* th = theta + (size_t)b * P + LEAD;
  int k = 0;
  const dd sig2 = space == 0 ? dd_exp(dd_make(th[k])) : dd_make(th[k]);
  ++k;
  dd U[M][M];
#pragma unroll
  for (int j = 0; j < M; ++j)
#pragma unroll
    for (int i = 0; i < M; ++i) {
      if (i <= j) {
        const double x = th[k++];
        U[i][j] = (i == j && space == 0) ? dd_exp(dd_make(x)) : dd_make(x);
      } else {
        U[i][j] = dd_make(0.0);
      }
    }
  dd Q[M][M];
#pragma unroll
  for (int i = 0; i < M; ++i)
#pragma unroll
    for (int j = 0; j < M; ++j) {
      dd_acc a;
#pragma unroll
      for (int l = 0; l < M; ++l) a.add_prod(U[l][i], U[l][j]);  // Q = U'U (paramoperations.jl:35)
      Q[i][j] = a.value();
    }
  double delta[M];
#pragma unroll
  for (int i = 0; i < M; ++i) delta[i] = th[k++];
  dd Phi[M][M];
#pragma unroll
  for (int i = 0; i < M; ++i)
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const double x = th[k++];
      Phi[i][j] = (i == j && space == 0) ? dd_from_R_to_11(x) : dd_make(x);  // row-major (paramoperations.jl:38)
    }
  // β₀ = (I − Φ) \ δ
  dd A[M][M], x[M][1];
#pragma unroll
  for (int i = 0; i < M; ++i) {
#pragma unroll
    for (int j = 0; j < M; ++j) A[i][j] = (i == j) ? dd_add_d(dd_neg(Phi[i][j]), 1.0) : dd_neg(Phi[i][j]);
    x[i][0] = dd_make(delta[i]);
  }
  bool ok = dd_gauss<M, 1>(A, x);
  // P₀: the M(M+1)/2 unknowns P_ij (i ≤ j) of P − ΦPΦ' = Q (singular iff I − Φ⊗Φ is)
  constexpr int S = R::U;
  dd Ls[S][S], qv[S][1];
  int rr = 0;
#pragma unroll
  for (int i = 0; i < M; ++i)
#pragma unroll
    for (int j = i; j < M; ++j) {
      int c = 0;
#pragma unroll
      for (int kk = 0; kk < M; ++kk)
#pragma unroll
        for (int l = kk; l < M; ++l) {
          dd s = dd_mul(Phi[i][kk], Phi[j][l]);
          if (kk != l) s = dd_add(s, dd_mul(Phi[i][l], Phi[j][kk]));
          Ls[rr][c] = (rr == c) ? dd_add_d(dd_neg(s), 1.0) : dd_neg(s);
          ++c;
        }
      qv[rr][0] = Q[i][j];
      ++rr;
    }
  ok = dd_gauss<S, 1>(Ls, qv) && ok;
  r[R::Sig] = sig2.hi;
  r[R::Sig + 1] = sig2.lo;
  int q = 0;
#pragma unroll
  for (int i = 0; i < M; ++i) {
    r[R::Delta + i] = delta[i];
    r[R::Beta + 2 * i] = x[i][0].hi;
    r[R::Beta + 2 * i + 1] = x[i][0].lo;
#pragma unroll
    for (int j = 0; j < M; ++j) {
      r[R::Phi + 2 * (i * M + j)] = Phi[i][j].hi;
      r[R::Phi + 2 * (i * M + j) + 1] = Phi[i][j].lo;
    }
#pragma unroll
    for (int j = i; j < M; ++j, ++q) {
      r[R::Q + 2 * q] = Q[i][j].hi;
      r[R::Q + 2 * q + 1] = Q[i][j].lo;
      r[R::P0 + 2 * q] = qv[q][0].hi;
      r[R::P0 + 2 * q + 1] = qv[q][0].lo;
    }
  }
  r[R::Ok] = ok ? 1.0 : 0.0;
  r[R::Ok + 1] = 0.0;
  }
}

template <int M, int LEAD>
__device__ __noinline__ void fd_init_record_call(const double* __restrict__ theta, int P, int space, int b,
                                                 double* __restrict__ r) {
  fd_init_record<M, LEAD>(theta, P, space, b, r);
}

template <int L, int M, int LEAD, bool RECORD>
__global__ __launch_bounds__(kFdBlock) void fixedz_dd_loglik_kernel(
    double* __restrict__ rec, const int* __restrict__ defer_list, const int* __restrict__ defer_count,
    const double* __restrict__ theta, int P, int space, const double* __restrict__ Y, const double* __restrict__ prep, int ldp,
    int np, int T, int N, int TC, const double* __restrict__ mats, const int* __restrict__ T_use,
    double* __restrict__ out, unsigned int* __restrict__ flags, double* __restrict__ rec_beta,
    double* __restrict__ rec_P, int horizon, int rec_len) {
  using R = FdRec<M>;
  constexpr int U = R::U;
  constexpr int NZ = M - 1;
  constexpr int GPB = kFdBlock / L;
  constexpr int MPL = (M >= 5 ? 8 : 16);  // maturities per lane: N ≤ MPL·L (as yfm_group.hip)
  static_assert(NZ == 2 * LEAD, "loading columns come in (S, C) pairs per gamma");
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* s_nan = smem;             // TC NaN flags of the staged chunk
  double* s_y = smem + TC;          // TC columns of N yields
  double* s_par = s_y + TC * N;     // per group: σ², δ, Φ, Q (R::Par doubles)
  __shared__ int s_nobs_max;

  const int nd = *defer_count;
  const int tid = threadIdx.x;
  const int j = tid % L;
  const int grp = tid / L;
  // a small grid walks the deferral list (the list is usually empty: the launch must cost ~nothing)
  for (int base = blockIdx.x * GPB; base < nd; base += gridDim.x * GPB) {  // block-uniform bound
  const int g = base + grp;
  const bool live = g < nd;
  // an idle group reads the record of this block's first group (base < nd: written above by this same
  // workgroup before the barrier), never one another block may still be writing
  const int gg = live ? g : base;
  const int b = defer_list[gg];
  const int nobs = T_use ? T_use[b] : T;

  if (tid == 0) s_nobs_max = 0;
  if (live && j == 0) {
    if constexpr (M == 3)
      fd_init_record<M, LEAD>(theta, P, space, b, rec + (size_t)gg * R::Len);
    else
      fd_init_record_call<M, LEAD>(theta, P, space, b, rec + (size_t)gg * R::Len);
  }
  __syncthreads();  // the record (global memory, this workgroup) before its lanes read it
  const double* r = rec + (size_t)gg * R::Len;
  double* par = s_par + grp * R::Par;
  for (int q = j; q < R::Par; q += L) par[q] = r[q];
  __syncthreads();
  const int my_steps = horizon > 0 ? nobs + horizon : nobs - 1;  // as yfm_kernels.hip
  const int my_data = horizon > 0 ? nobs : nobs - 1;
  atomicMax(&s_nobs_max, live ? my_steps : 0);

  // this lane's loadings in dd (dns.jl:51-65): S = (1 − e^{−λm})/(λm), C = S − e^{−λm}
  dd Zl[MPL][NZ];
  dd_acc gacc[NZ + NZ * (NZ + 1) / 2];
#pragma unroll
  for (int l = 0; l < LEAD; ++l) {
    const dd lam = dd_add_d(dd_exp(dd_make(theta[(size_t)b * P + l])), 1e-2);  // dns.jl:55
    const bool finite_lam = lam.hi < __builtin_inf();
#pragma unroll
    for (int k = 0; k < MPL; ++k) {
      const int i = j + k * L;
      dd s = dd_make(0.0), c = dd_make(0.0);
      if (i < N && finite_lam) {
        const double m = mats[i];
        const dd tau = dd_mul_d(lam, m);
        const dd z = dd_exp(neg_rate(lam, m));
        if (tau.hi < __builtin_inf()) {
          s = dd_div(dd_add_d(dd_neg(z), 1.0), tau);
          c = dd_sub(s, z);
        }
      }
      // (λ = Inf: FP64 gives S = 1/Inf = 0, C = 0 − 0; kept)
      Zl[k][2 * l] = s;
      Zl[k][2 * l + 1] = c;
    }
  }
#pragma unroll
  for (int k = 0; k < MPL; ++k) {
    int q = NZ;
#pragma unroll
    for (int c = 0; c < NZ; ++c) {
      gacc[c].add(Zl[k][c]);
#pragma unroll
      for (int d = c; d < NZ; ++d, ++q) gacc[q].add_prod(Zl[k][c], Zl[k][d]);
    }
  }
  dd G[M][M];
  G[0][0] = dd_make((double)N);
  {
    int q = NZ;
#pragma unroll
    for (int c = 0; c < NZ; ++c) {
      G[0][c + 1] = G[c + 1][0] = group_sum_acc<L>(gacc[c]);
#pragma unroll
      for (int d = c; d < NZ; ++d, ++q) G[c + 1][d + 1] = G[d + 1][c + 1] = group_sum_acc<L>(gacc[q]);
    }
  }

  dd beta[M], Pm[U];
#pragma unroll
  for (int i = 0; i < M; ++i) beta[i] = {r[R::Beta + 2 * i], r[R::Beta + 2 * i + 1]};
#pragma unroll
  for (int q = 0; q < U; ++q) Pm[q] = {r[R::P0 + 2 * q], r[R::P0 + 2 * q + 1]};
  const bool init_ok = r[R::Ok] != 0.0;
  const dd sig2 = {par[R::Sig], par[R::Sig + 1]};
  const dd rsig2 = dd_rcp(sig2);

  dd_acc sum_ld, sum_q;
  bool neg = false;
  double last_ld = -__builtin_inf(), last_q = 0.0;  // fresh model: F = 0 (logdet −Inf), v = 0
  bool last_neg = false;

  __syncthreads();
  const int nsteps = max(s_nobs_max, 0);
  const int CHY = TC * N;

  double pre[kFdPre];
  double pre_nan = 0.0;
  auto load_chunk = [&](int c) {
    const size_t base = (size_t)c * CHY;
    const size_t lim = (size_t)T * N;
#pragma unroll
    for (int q = 0; q < kFdPre; ++q) {
      const int e = q * kFdBlock + tid;
      const size_t gi = base + e;
      pre[q] = (e < CHY && gi < lim) ? Y[gi] : 0.0;
    }
    const int tc = c * TC + tid;
    pre_nan = (tid < TC && tc < T) ? prep[(size_t)tc * ldp + np + 2] : 0.0;
  };
  auto store_chunk = [&]() {
#pragma unroll
    for (int q = 0; q < kFdPre; ++q) {
      const int e = q * kFdBlock + tid;
      if (e < CHY) s_y[e] = pre[q];
    }
    if (tid < TC) s_nan[tid] = pre_nan;
  };
  if (nsteps > 0) {
    load_chunk(0);
    store_chunk();
    __syncthreads();
    load_chunk(1);
  }

  for (int t = 0; t < nsteps; ++t) {
    const int tt = t % TC;
    const bool act = live && t < my_steps;
    const bool acc = t >= 1;  // Julia t > 1 (filter.jl:194)
    const bool nan_col = s_nan[tt] != 0.0 || t >= my_data;
    if (act && nan_col) {
      // filter.jl:126-140: prediction only; F, F⁻¹, v stale → the loglik re-adds the last term
      dd bf[M], X[U];
#pragma unroll
      for (int i = 0; i < M; ++i) bf[i] = beta[i];
#pragma unroll
      for (int q = 0; q < U; ++q) X[q] = Pm[q];
      fd_propagate<M>(par, bf, X, false, beta, Pm);
      if (acc) {
        sum_ld.add(dd_make(last_ld));
        sum_q.add(dd_make(last_q));
        neg = neg || last_neg;
      }
    } else if (act) {
      // the innovation per owned maturity (filter.jl:143-144) and its sums u = Z'v, v'v
      const double* col = s_y + tt * N;
      dd_acc ua[M], va;
#pragma unroll
      for (int k = 0; k < MPL; ++k) {
        const int i = j + k * L;
        if (i < N) {
          dd_acc yh;
          yh.add(beta[0]);
#pragma unroll
          for (int c = 0; c < NZ; ++c) yh.add_prod(Zl[k][c], beta[c + 1]);
          const dd v = dd_add_d(dd_neg(yh.value()), col[i]);
          ua[0].add(v);
#pragma unroll
          for (int c = 0; c < NZ; ++c) ua[c + 1].add_prod(Zl[k][c], v);
          va.add_prod(v, v);
        }
      }
      dd u[M];
#pragma unroll
      for (int c = 0; c < M; ++c) u[c] = group_sum_acc<L>(ua[c]);
      const dd vv = group_sum_acc<L>(va);
      // capacitance solve: B̃ = σ²I + P G, W = B̃⁻¹P (symmetric part)
      dd A[M][M], W[M][M];
#pragma unroll
      for (int i = 0; i < M; ++i)
#pragma unroll
        for (int c = 0; c < M; ++c) {
          dd_acc a;
          if (i == c) a.add(sig2);
#pragma unroll
          for (int l = 0; l < M; ++l) a.add_prod(Pm[us<M>(i, l)], G[l][c]);
          A[i][c] = a.value();
          W[i][c] = Pm[us<M>(i, c)];
        }
      dd det;
      dd_gauss<M, M>(A, W, &det);
      dd Ws[U];
#pragma unroll
      for (int i = 0; i < M; ++i)
#pragma unroll
        for (int c = i; c < M; ++c) Ws[ut<M>(i, c)] = (i == c) ? W[i][i] : dd_ldexp(dd_add(W[i][c], W[c][i]), -1);
      dd bf[M];
      dd_acc uk;
#pragma unroll
      for (int i = 0; i < M; ++i) {
        dd_acc a;
#pragma unroll
        for (int c = 0; c < M; ++c) a.add_prod(Ws[us<M>(i, c)], u[c]);
        const dd kv = a.value();
        bf[i] = dd_add(beta[i], kv);
        uk.add_prod(u[i], kv);
      }
      const double q = dd_to_double(dd_mul(dd_sub(vv, uk.value()), rsig2));
      const double dh = dd_to_double(det);
      const bool upd = dh != 0.0;  // inv(F) threw: no update (filter.jl:151-154)
      if (upd) fd_propagate<M>(par, bf, Ws, true, beta, Pm);
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
      // the state after step t into slot t − max(0, my_steps − rec_len) (FixedZFilter::record)
      const int slot = t - max(0, my_steps - rec_len);
      if (act && j == 0 && slot >= 0) {
        const size_t o = (size_t)b * (size_t)rec_len + slot;
#pragma unroll
        for (int i = 0; i < M; ++i) rec_beta[o * M + i] = dd_to_double(beta[i]);
        if (rec_P) {
#pragma unroll
          for (int c = 0; c < M; ++c)
#pragma unroll
            for (int i = 0; i < M; ++i) rec_P[o * M * M + c * M + i] = dd_to_double(Pm[us<M>(i, c)]);
        }
      }
    }
    if (tt == TC - 1) {
      __syncthreads();
      store_chunk();
      __syncthreads();
      load_chunk(t / TC + 2);
    }
  }

  if (live && j == 0) {
  atomicAdd(&flags[3], 1u);  // n_deferred (yfm_last_batch_deferred)
  double ll;
  if (!init_ok) {
    ll = __builtin_nan("");  // the reference throws from initialize_filter
    atomicAdd(&flags[0], 1u);
  } else {
    const int nterms = max(nobs - 2, 0);
    if (nterms == 0) {
      ll = 0.0;
    } else {
      // per term: (N − M)·log σ² + N·log 2π (+ log|det B̃_t| + q_t, summed above)
      const dd lsig = dd_log(sig2);
      dd tot = dd_mul_d(dd_add_d(dd_mul_d(lsig, (double)(N - M)), (double)N * kLog2Pi), (double)nterms);
      tot = dd_add(tot, dd_add(sum_ld.value(), sum_q.value()));
      ll = -0.5 * dd_to_double(tot);
    }
    if (neg || !isfinite(ll)) {  // DomainError / non-finite → -Inf (filter.jl:197-204)
      ll = -__builtin_inf();
      atomicAdd(&flags[1], 1u);
    }
  }
  out[b] = ll;
  }
  __syncthreads();  // LDS (panel chunks, per-group parameters) reused by the next slot group
  }
}

namespace {

template <int L, int M, int LEAD>
hipError_t launch_fd_l(const LaunchArgs& a, double* rec, int TC) {
  constexpr int GPB = kFdBlock / L;
  const int grid = std::min((a.B + GPB - 1) / GPB, 256);
  const size_t shmem = sizeof(double) * ((size_t)TC + (size_t)TC * a.N + (size_t)GPB * FdRec<M>::Par);
  if (shmem > 64 * 1024) return hipErrorInvalidValue;
  if (a.rec_beta) {
    hipLaunchKernelGGL((fixedz_dd_loglik_kernel<L, M, LEAD, true>), dim3(grid), dim3(kFdBlock), shmem, a.stream, rec,
                       a.defer_list, a.defer_count, a.theta, a.P, a.space, a.raw, a.panel, a.ldp, a.np, a.T, a.N, TC, a.mats,
                       a.T_use, a.out, a.flags, a.rec_beta, a.rec_P, a.horizon, a.rec_len);
  } else {
    hipLaunchKernelGGL((fixedz_dd_loglik_kernel<L, M, LEAD, false>), dim3(grid), dim3(kFdBlock), shmem, a.stream, rec,
                       a.defer_list, a.defer_count, a.theta, a.P, a.space, a.raw, a.panel, a.ldp, a.np, a.T, a.N, TC, a.mats,
                       a.T_use, a.out, a.flags, nullptr, nullptr, 0, 0);
  }
  return hipGetLastError();
}

template <int M, int LEAD>
hipError_t launch_fd_m(const LaunchArgs& a, double* rec) {
  constexpr int MPL = M >= 5 ? 8 : 16;
  int L = 4;
  while (L * MPL < a.N && L < 64) L <<= 1;
  if (L * MPL < a.N) return hipErrorInvalidValue;
  int TC = (kFdPre * kFdBlock) / a.N;
  if (TC > 32) TC = 32;
  if (TC < 1) return hipErrorInvalidValue;
  switch (L) {
    case 4: return launch_fd_l<4, M, LEAD>(a, rec, TC);
    case 8: return launch_fd_l<8, M, LEAD>(a, rec, TC);
    case 16: return launch_fd_l<16, M, LEAD>(a, rec, TC);
    case 32: return launch_fd_l<32, M, LEAD>(a, rec, TC);
    case 64: return launch_fd_l<64, M, LEAD>(a, rec, TC);
  }
  return hipErrorInvalidValue;
}

}  // namespace

size_t fixedz_dd_scratch_bytes(int kind, int B) {
  const size_t len = kind == 2 ? FdRec<5>::Len : FdRec<3>::Len;
  return sizeof(double) * len * (size_t)(B > 0 ? B : 1);
}

hipError_t launch_fixedz_dd(int kind, const LaunchArgs& a, double* rec) {
  if (!a.defer_list || !a.defer_count || !rec) return hipErrorInvalidValue;
  if (kind == 0) return launch_fd_m<3, 1>(a, rec);
  if (kind == 2) return launch_fd_m<5, 2>(a, rec);
  return hipErrorInvalidValue;
}

}  // namespace yfm

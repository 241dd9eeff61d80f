// yfm_group.hip — fixed-loading models (DNS, GNS5) for maturity counts beyond the
// one-filter-per-lane kernel's register budget (N > 64, e.g. the 360 monthly maturities of
// config 3's panel): ONE FILTER PER GROUP OF L LANES.
//
// Restates the same reference functions as yfm_kernels.hip (get_loss filter.jl:182-209,
// filter! filter.jl:125-179, initialize_filter filter.jl:1-10, dns.jl:51-65), through the
// shared collapsed-form filter (yfm_fixedz.hpp).  Only z̃_t = Z'ỹ_t is formed differently:
// lane j of a group owns the maturities i ≡ j (mod L) and their loadings (≤ kGMaxPL per lane,
// in VGPRs for the whole filter), forms its partial dot products against the staged panel
// column and the group reduces them with DPP / permlane butterflies (group_sum, no LDS).
// Z'Z is formed the same way once.  Every lane of the group then runs the M×M update
// redundantly, so the state stays replicated and no broadcast is needed; lane 0 writes.
// Candidates with an ill-conditioned Z'Z are appended to the deferral list (as in the per-lane
// kernel) for the double-double capacitance kernel (yfm_fixedz_dd.hip).
//
// Panel: the prepared centered panel (prep_panel_kernel layout, ldp doubles per column),
// TC columns per LDS chunk, the next chunk prefetched into registers (as yfm_tvl.hip).
#include "yfm_fixedz.hpp"
#include "yfm_internal.hpp"

namespace yfm {

namespace {

constexpr int kGBlock = 256;
constexpr int kGPre = 8;  // prepared-panel doubles prefetched per thread per chunk

template <int M>
constexpr int group_max_per_lane() {
  return M >= 5 ? 8 : 16;  // maturities per lane: N ≤ kGMaxPL · L
}

}  // namespace

template <int L, int M, int LEAD, bool RECORD>
__global__ __launch_bounds__(kGBlock, 2) void fixedz_group_kernel(
    const double* __restrict__ theta, int P, int B, int space, const double* __restrict__ panel, int ldp, int np,
    int T, int N, int TC, const double* __restrict__ mats, const int* __restrict__ T_use, double* __restrict__ out,
    unsigned int* __restrict__ flags, double* __restrict__ rec_beta, double* __restrict__ rec_P, int horizon,
    int rec_len, int* __restrict__ defer_list, int* __restrict__ defer_count, unsigned int* __restrict__ flags_next) {
  if (flags_next && blockIdx.x == 0 && threadIdx.x < kFlagsPerBank) flags_next[threadIdx.x] = 0u;  // the next launch's counters
  constexpr int NZ = M - 1;
  constexpr int GPB = kGBlock / L;  // filters per block
  constexpr int MPL = group_max_per_lane<M>();
  constexpr int NG = NZ + NZ * (NZ + 1) / 2;  // Σ Z_c and Σ Z_c Z_d (c ≤ d)
  static_assert(NZ == 2 * LEAD, "loading columns come in (S, C) pairs per gamma");
  extern __shared__ __attribute__((aligned(16))) double s_col[];  // TC × ldp
  __shared__ int s_nobs_max;

  const int tid = threadIdx.x;
  const int j = tid % L;
  const int b = blockIdx.x * GPB + tid / L;
  const bool live = b < B;
  const int bb = live ? b : B - 1;
  const int nobs = T_use ? T_use[bb] : T;
  const int my_steps = horizon > 0 ? nobs + horizon : nobs - 1;  // as yfm_kernels.hip
  const int my_data = horizon > 0 ? nobs : nobs - 1;

  if (tid == 0) s_nobs_max = 0;
  __syncthreads();
  atomicMax(&s_nobs_max, live ? my_steps : 0);

  FixedZFilter<M, LEAD, RECORD> f;
  decode_params<M, LEAD>(theta + (size_t)bb * P, space, f.p);

  // this lane's loadings (dns.jl:51-65; the GNS5 extension adds a second (S, C) pair)
  double Zl[MPL][NZ];
  double gs[NG];
#pragma unroll
  for (int k = 0; k < NG; ++k) gs[k] = 0.0;
#pragma unroll
  for (int k = 0; k < MPL; ++k) {
    const int i = j + k * L;
    const bool own = i < N;
    const double m = own ? mats[i] : 1.0;
#pragma unroll
    for (int l = 0; l < LEAD; ++l) {
      const double lam = 1e-2 + exp(f.p.gam[l]);  // dns.jl:55
      const double tau = lam * m;
      const double z = exp(-tau);
      const double s = (1.0 - z) / tau;
      Zl[k][2 * l] = own ? s : 0.0;
      Zl[k][2 * l + 1] = own ? s - z : 0.0;
    }
    int q = NZ;
#pragma unroll
    for (int c = 0; c < NZ; ++c) {
      gs[c] += Zl[k][c];
#pragma unroll
      for (int d = c; d < NZ; ++d, ++q) gs[q] = fma(Zl[k][c], Zl[k][d], gs[q]);
    }
  }
#pragma unroll
  for (int k = 0; k < NG; ++k) gs[k] = group_sum<L>(gs[k]);
  double G[M][M];
  G[0][0] = (double)N;
  {
    int q = NZ;
#pragma unroll
    for (int c = 0; c < NZ; ++c) {
      G[0][c + 1] = G[c + 1][0] = gs[c];
#pragma unroll
      for (int d = c; d < NZ; ++d, ++q) G[c + 1][d + 1] = G[d + 1][c + 1] = gs[q];
    }
  }
  f.setup(G, N);
  const bool defer = live && !f.collapsed;
  if (defer && j == 0) defer_list[atomicAdd(defer_count, 1)] = b;

  __syncthreads();
  const int nsteps = max(s_nobs_max, 0);
  const int CH = TC * ldp;  // doubles per chunk

  // ---- panel staging: chunk c in LDS, chunk c+1 in registers ------------------------------
  double pre[kGPre];
  auto load_chunk = [&](int c) {
    const size_t base = (size_t)c * CH;
    const size_t lim = (size_t)T * ldp;
#pragma unroll
    for (int r = 0; r < kGPre; ++r) {
      const int e = r * kGBlock + tid;
      const size_t g = base + e;
      pre[r] = (e < CH && g < lim) ? panel[g] : 0.0;
    }
  };
  auto store_chunk = [&]() {
#pragma unroll
    for (int r = 0; r < kGPre; ++r) {
      const int e = r * kGBlock + tid;
      if (e < CH) s_col[e] = pre[r];
    }
  };
  if (nsteps > 0) {
    load_chunk(0);
    store_chunk();
    __syncthreads();
    load_chunk(1);
  }

  for (int t = 0; t < nsteps; ++t) {
    const int tt = t % TC;
    const double* col = s_col + tt * ldp;
    double zc[NZ];
#pragma unroll
    for (int c = 0; c < NZ; ++c) zc[c] = 0.0;
#pragma unroll
    for (int k = 0; k < MPL; ++k) {
      const int i = j + k * L;
      const double y = (i < np) ? col[i] : 0.0;  // ỹ is zero-padded up to np
#pragma unroll
      for (int c = 0; c < NZ; ++c) zc[c] = fma(Zl[k][c], y, zc[c]);
    }
#pragma unroll
    for (int c = 0; c < NZ; ++c) zc[c] = group_sum<L>(zc[c]);
    const double2 yb = *reinterpret_cast<const double2*>(col + np);
    const double2 meta = *reinterpret_cast<const double2*>(col + np + 2);
    f.step(t, zc, yb, meta, false, my_steps, my_data);
    if constexpr (RECORD) {
      if (live && !defer && j == 0) f.record(t, b, my_steps, rec_len, rec_beta, rec_P);
    }
    if (tt == TC - 1) {  // chunk done: its buffer takes the prefetched chunk, prefetch the one after
      __syncthreads();
      store_chunk();
      __syncthreads();
      load_chunk(t / TC + 2);
    }
  }

  if (!live || defer || j != 0) return;
  out[b] = f.loglik(nobs, flags);
}

namespace {

template <int L, int M, int LEAD>
hipError_t launch_group_l(const LaunchArgs& a, int TC) {
  constexpr int GPB = kGBlock / L;
  const int grid = (a.B + GPB - 1) / GPB;
  const size_t shmem = sizeof(double) * (size_t)TC * a.ldp;
  if (a.rec_beta) {
    hipLaunchKernelGGL((fixedz_group_kernel<L, M, LEAD, true>), dim3(grid), dim3(kGBlock), shmem, a.stream, a.theta,
                       a.P, a.B, a.space, a.panel, a.ldp, a.np, a.T, a.N, TC, a.mats, a.T_use, a.out, a.flags,
                       a.rec_beta, a.rec_P, a.horizon, a.rec_len, a.defer_list, a.defer_count, a.flags_next);
  } else {
    hipLaunchKernelGGL((fixedz_group_kernel<L, M, LEAD, false>), dim3(grid), dim3(kGBlock), shmem, a.stream, a.theta,
                       a.P, a.B, a.space, a.panel, a.ldp, a.np, a.T, a.N, TC, a.mats, a.T_use, a.out, a.flags,
                       nullptr, nullptr, 0, 0, a.defer_list, a.defer_count, a.flags_next);
  }
  return hipGetLastError();
}

template <int M, int LEAD>
hipError_t launch_group_m(const LaunchArgs& a, int L, int TC) {
  switch (L) {
    case 4: return launch_group_l<4, M, LEAD>(a, TC);
    case 8: return launch_group_l<8, M, LEAD>(a, TC);
    case 16: return launch_group_l<16, M, LEAD>(a, TC);
    case 32: return launch_group_l<32, M, LEAD>(a, TC);
    case 64: return launch_group_l<64, M, LEAD>(a, TC);
  }
  return hipErrorInvalidValue;
}

}  // namespace

int group_max_n(int kind) { return 64 * (kind == 2 ? group_max_per_lane<5>() : group_max_per_lane<3>()); }

int group_lanes_for(int kind, int N) {
  const int mpl = kind == 2 ? group_max_per_lane<5>() : group_max_per_lane<3>();
  int L = 4;
  while (L * mpl < N && L < 64) L <<= 1;
  return L * mpl >= N ? L : -1;
}

hipError_t launch_fixedz_group(int kind, const LaunchArgs& a) {
  if (!a.defer_list || !a.defer_count) return hipErrorInvalidValue;
  const int L = group_lanes_for(kind, a.N);
  if (L < 0) return hipErrorInvalidValue;
  int TC = (kGPre * kGBlock) / a.ldp;  // columns per chunk: the prefetch registers hold ≤ kGPre·256
  if (TC > 32) TC = 32;
  if (TC < 1) return hipErrorInvalidValue;
  if (kind == 0) return launch_group_m<3, 1>(a, L, TC);
  if (kind == 2) return launch_group_m<5, 2>(a, L, TC);
  return hipErrorInvalidValue;
}

}  // namespace yfm

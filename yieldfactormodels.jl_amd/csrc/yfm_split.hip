// yfm_split.hip — the DNS batched log-likelihood with each filter split over TWO WAVES
// (the headline configuration: N ≤ 32 maturities, M = 3).
//
// Restates the same reference functions as yfm_kernels.hip — get_loss (filter.jl:182-209),
// filter! (filter.jl:125-179), initialize_filter (filter.jl:1-10), the DNS loadings
// (dns.jl:51-65), transform_params / set_params! — with the same per-value arithmetic as the
// one-filter-per-lane kernel (yfm_fixedz.hpp: collapsed_cov + collapsed_mean), so the two give
// the same bits; only the schedule differs.
//
// Why: at the headline batch (65,536 θ) one filter per lane is exactly one wave per SIMD, and the
// M×M recursion of a single wave leaves ~45% of the FP64 issue slots empty on dependency stalls
// (PMC).  The collapsed form separates into two recursions:
//   covariance (data-independent): P_t → S_t = P_t + R → LDLᵀ(S_t), det S_t → P_{t|t} = P S⁻¹R
//                                   → P_{t+1} = ΦP_{t|t}Φ' + Q;
//   mean / loglik:                 z̃_t = Z'ỹ_t (MFMA) → ĉ, ‖ỹ − Zĉ‖² → x = S_t⁻¹(ĉ − β) →
//                                   q, β_{t|t} = β + P_t x → β_{t+1} = δ + Φβ_{t|t}.
// A block of 512 threads holds 4 COVARIANCE waves and 4 MEAN waves for the same 256 candidates
// (lane l of covariance wave w and of mean wave w own the same candidate), i.e. two instruction
// streams per SIMD.  In iteration k the covariance wave produces step k's factor record
// (L, 1/d, P_t, det S_t — 13 doubles per candidate) into an LDS ring while the mean wave consumes
// step k − 1's; one workgroup barrier per iteration orders them (2 ring slots).
//
// Trajectory mode (predict / filter_states): the mean wave records β, the covariance wave P.
// Ill-conditioned Z'Z lanes are deferred to the double-double kernel exactly as in the per-lane
// kernel (both waves compute the same decision).
#include "yfm_fixedz.hpp"
#include "yfm_internal.hpp"

#include <cstdlib>
#include <type_traits>

namespace yfm {

namespace {

constexpr int kSplitBlock = 512;  // 4 covariance + 4 mean waves
constexpr int kSplitPairs = 4;
constexpr int kSTC = 32;          // panel columns per LDS chunk
constexpr int kSTB = 16;          // steps per MFMA block
constexpr int kRec = 13;          // L10 L20 L21, 1/d0..2, P00 P01 P02 P11 P12 P22, det S

}  // namespace

template <int NP, bool RECORD>
__global__ __launch_bounds__(kSplitBlock, 1) void dns_split_kernel(
    const double* __restrict__ theta, int P, int B, int space, const double* __restrict__ panel, int T, int N,
    const double* __restrict__ mats, const int* __restrict__ T_use, double* __restrict__ out,
    unsigned int* __restrict__ flags, double* __restrict__ rec_beta, double* __restrict__ rec_P, int horizon,
    int rec_len, int* __restrict__ defer_list, int* __restrict__ defer_count, int interleave,
    unsigned int* __restrict__ flags_next) {
  constexpr int M = 3, LEAD = 1, NZ = 2;
  if (flags_next && blockIdx.x == 0 && threadIdx.x < kFlagsPerBank) flags_next[threadIdx.x] = 0u;  // the next launch's counters
  constexpr int LDP = NP + 4;
  constexpr int CH = kSTC * LDP;
  constexpr int PER = (CH + kSplitBlock - 1) / kSplitBlock;
  constexpr int NK = (NP + 3) / 4;     // MFMA k-steps
  constexpr int NRT = 64 * NZ / 16;    // MFMA row tiles per wave
  constexpr int SS = 64 * NZ + 2;      // scratch row stride (doubles)
  constexpr int SCR = kSTB * SS;
  static_assert(NP <= 32 && NP % 2 == 0, "MFMA fragments and double2 panel reads");
  __shared__ __attribute__((aligned(16))) double sh[2][CH];
  __shared__ __attribute__((aligned(16))) double scratch[kSplitPairs][SCR];
  __shared__ double ring[2][kSplitPairs][kRec][64];
  __shared__ int s_nobs_max;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  // interleave 0: waves 0-3 covariance, 4-7 mean; 1: even waves covariance, odd waves mean
  const bool cov = interleave ? !(wave & 1) : wave < kSplitPairs;
  const int pair = interleave ? (wave >> 1) : (wave & (kSplitPairs - 1));
  const int b = blockIdx.x * (kSplitPairs * 64) + pair * 64 + lane;
  const bool live = b < B;
  const int bb = live ? b : (B - 1);
  const int nobs = T_use ? T_use[bb] : T;

  if (tid == 0) s_nobs_max = 0;
  __syncthreads();
  const int my_steps = horizon > 0 ? nobs + horizon : nobs - 1;  // as yfm_kernels.hip
  const int my_data = horizon > 0 ? nobs : nobs - 1;
  atomicMax(&s_nobs_max, live ? my_steps : 0);

  // The two roles run disjoint code (their register live ranges never meet): the covariance wave's
  // M×M state and the mean wave's MFMA fragments each fit the 256 registers of two waves per SIMD.
  auto role = [&](auto is_cov) {
    constexpr bool COV = decltype(is_cov)::value;
  // ---- decode θ_b, loadings, Z'Z, initial state (both roles, same arithmetic) ----------------
  FixedZFilter<M, LEAD, RECORD> f;
  decode_params<M, LEAD>(theta + (size_t)bb * P, space, f.p);
  const double lam = 1e-2 + exp(f.p.gam[0]);  // dns.jl:55
  // loading pair (S, C) at maturity i (zero past N): S = (1 − e^{−λm})/(λm), C = S − e^{−λm}
  auto loading = [&](int i, double& s, double& c) {
    if (i < N) {
      const double tau = lam * mats[i];
      const double z = exp(-tau);
      s = (1.0 - z) / tau;
      c = s - z;
    } else {
      s = 0.0;
      c = 0.0;
    }
  };
  // Z'Z summed in maturity order (the per-lane kernel's order, so both kernels defer the same lanes)
  double G[M][M];
  double gs[NZ] = {0.0, 0.0}, gg[3] = {0.0, 0.0, 0.0};
  auto acc_gram = [&](double s, double c) {
    gs[0] += s;
    gs[1] += c;
    gg[0] = fma(s, s, gg[0]);
    gg[1] = fma(s, c, gg[1]);
    gg[2] = fma(c, c, gg[2]);
  };
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    double zs, zc;
    loading(i, zs, zc);
    acc_gram(zs, zc);
  }
  G[0][0] = (double)N;
  G[0][1] = G[1][0] = gs[0];
  G[0][2] = G[2][0] = gs[1];
  G[1][1] = gg[0];
  G[1][2] = G[2][1] = gg[1];
  G[2][2] = gg[2];
  f.setup(G, N, true);  // before the fragments: its solves' registers must not coexist with them
  const bool defer = live && !f.collapsed;
  if constexpr (!COV) {
    if (defer) defer_list[atomicAdd(defer_count, 1)] = b;
  }
  // MFMA A fragments (mean waves): tile r, k-step kk — lane l holds Z of pair p = 16r + (l & 15)
  // (candidate p >> 1 of this wave, column p & 1) at maturity 4kk + (l >> 4); staged through the
  // wave's scratch one quarter (16 candidates) at a time, each lane writing its own loadings
  double Af[COV ? 1 : NRT][COV ? 1 : NK];
  if constexpr (!COV) {
    constexpr int ZS = 4 * NK + 1;
    constexpr int QT = NRT / 4;
    static_assert(16 * NZ * ZS <= SCR, "staging fits the scratch");
    double* st = scratch[pair];
#pragma unroll
    for (int qu = 0; qu < 4; ++qu) {
      if ((lane >> 4) == qu) {
        const int cl = lane & 15;
#pragma unroll
        for (int m = 0; m < ZS; ++m) {
          double zs, zc;
          loading(m < NP ? m : NP, zs, zc);
          st[(cl * NZ + 0) * ZS + m] = zs;
          st[(cl * NZ + 1) * ZS + m] = zc;
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int r = qu * QT; r < (qu + 1) * QT; ++r) {
        const int pr = 16 * r + (lane & 15) - qu * 16 * NZ;
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) Af[r][kk] = st[pr * ZS + 4 * kk + (lane >> 4)];
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
  }

  int wmin = live ? my_data : 0x7fffffff;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) wmin = min(wmin, __shfl_xor(wmin, off));
  const int wave_min_data = __builtin_amdgcn_readfirstlane(wmin);

  __syncthreads();
  const int nsteps = max(s_nobs_max, 0);

  // ---- panel staging (all 512 threads): LDS holds chunks c and c+1 --------------------------
  double pre[PER];
  auto load_chunk = [&](int c) {
    const size_t base = (size_t)c * CH;
    const size_t lim = (size_t)T * LDP;
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      const int e = r * kSplitBlock + tid;
      const size_t g = base + e;
      pre[r] = (e < CH && g < lim) ? panel[g] : 0.0;
    }
  };
  auto store_chunk = [&](double* buf) {
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      const int e = r * kSplitBlock + tid;
      if (e < CH) buf[e] = pre[r];
    }
  };
  if (nsteps > 0) {
    load_chunk(0);
    store_chunk(sh[0]);
    load_chunk(1);
    store_chunk(sh[1]);
    __syncthreads();
    load_chunk(2);
  }
  auto col_of = [&](int t) -> const double* { return sh[(t / kSTC) & 1] + (t % kSTC) * LDP; };
  // end of iteration k (every wave, the same barriers): the mean waves finished chunk c = k/kSTC − 1,
  // whose buffer takes chunk c + 2
  // LDS-only workgroup barrier: orders the ring and the staged panel without waiting for the
  // panel prefetch still in flight from global memory (__syncthreads would wait for it every step)
  auto lds_barrier = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  };
  auto end_iteration = [&](int k) {
    lds_barrier();  // step k's record written / step k − 1's consumed
    if (k > 0 && k % kSTC == 0) {
      const int c = k / kSTC - 1;
      store_chunk(sh[c & 1]);
      lds_barrier();
      load_chunk(c + 3);
    }
  };
  auto phi = [&](int i, int j) { return f.p.Phi[i][j]; };

  if constexpr (COV) {
    // ==== covariance wave: step k in iteration k =============================================
    for (int k = 0; k <= nsteps; ++k) {
      const int t = k;
      if (t < nsteps) {
        const bool nan_col = col_of(t)[NP + 2] != 0.0;
        const bool fast = (t >= 1) && !nan_col && (t < wave_min_data);
        const bool act = t < my_steps;
        if (fast || (act && !nan_col && t < my_data)) {
          LDLT<M> fl;
          double Pf[M][M];
          const double det = collapsed_cov<M>(f.R, f.Pm, fl, Pf);
          double* slot = &ring[t & 1][pair][0][lane];
          slot[0 * 64] = fl.L[1][0];
          slot[1 * 64] = fl.L[2][0];
          slot[2 * 64] = fl.L[2][1];
          slot[3 * 64] = fl.rd[0];
          slot[4 * 64] = fl.rd[1];
          slot[5 * 64] = fl.rd[2];
          slot[6 * 64] = f.Pm[0][0];
          slot[7 * 64] = f.Pm[0][1];
          slot[8 * 64] = f.Pm[0][2];
          slot[9 * 64] = f.Pm[1][1];
          slot[10 * 64] = f.Pm[1][2];
          slot[11 * 64] = f.Pm[2][2];
          slot[12 * 64] = det;
          // (the per-lane kernel's rule: the fast loglik path propagates whatever det is)
          if ((fast && !RECORD) || det != 0.0) propagate_cov_f<M>(phi, f.p.Q, Pf, f.Pm);
        } else if (act) {
          // NaN column / forecast step: prediction only (filter.jl:126-140)
          double Pf[M][M];
#pragma unroll
          for (int i = 0; i < M; ++i)
#pragma unroll
            for (int j = i; j < M; ++j) Pf[i][j] = f.Pm[i][j];
          propagate_cov_f<M>(phi, f.p.Q, Pf, f.Pm);
        }
        if constexpr (RECORD) {
          const int rs = t - max(0, my_steps - rec_len);
          if (rec_P && live && !defer && act && rs >= 0) {
            const size_t o = (size_t)b * (size_t)rec_len + rs;
#pragma unroll
            for (int j = 0; j < M; ++j)
#pragma unroll
              for (int i = 0; i < M; ++i) rec_P[o * M * M + j * M + i] = f.Pm[i][j];
          }
        }
      }
      end_iteration(k);
    }
  } else {
  // ==== mean wave: step k − 1 in iteration k ==================================================
  double* scr = scratch[pair];
  for (int k = 0; k <= nsteps; ++k) {
    if (k >= 1) {
      const int t = k - 1;
      const int tt = t % kSTB;
      if (tt == 0) {
        // z̃ for steps t .. t+15 of all 64 candidates: NRT·NK MFMAs (v_mfma_f64_16x16x4_f64), row
        // tiles in two groups (bounds the live accumulators)
        const double* cb = col_of(t);
        double bvk[NK];
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
          const int m = 4 * kk + (lane >> 4);
          bvk[kk] = (m < NP) ? cb[(lane & 15) * LDP + m] : 0.0;
        }
        typedef double d4 __attribute__((ext_vector_type(4)));
        constexpr int RG = NRT / 4;
#pragma unroll
        for (int r0 = 0; r0 < NRT; r0 += RG) {
          d4 acc[RG];
#pragma unroll
          for (int r = 0; r < RG; ++r) acc[r] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int kk = 0; kk < NK; ++kk)
#pragma unroll
            for (int r = 0; r < RG; ++r)
              acc[r] = __builtin_amdgcn_mfma_f64_16x16x4f64(Af[r0 + r][kk], bvk[kk], acc[r], 0, 0, 0);
#pragma unroll
          for (int r = 0; r < RG; ++r)
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) scr[(lane & 15) * SS + 16 * (r0 + r) + (lane >> 4) + 4 * q4] = acc[r][q4];
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
      }
      const double* cb = col_of(t);
      const double2 z2 = *reinterpret_cast<const double2*>(scr + tt * SS + NZ * lane);
      const double zc[NZ] = {z2.x, z2.y};
      const double2 yb = *reinterpret_cast<const double2*>(cb + NP);
      const double2 meta = *reinterpret_cast<const double2*>(cb + NP + 2);
      const bool fast = (t >= 1) && (meta.x == 0.0) && (t < wave_min_data);
      const bool act = t < my_steps;
      if (fast || (act && meta.x == 0.0 && t < my_data)) {
        const double* slot = &ring[t & 1][pair][0][lane];
        LDLT<M> fl;
        fl.L[1][0] = slot[0 * 64];
        fl.L[2][0] = slot[1 * 64];
        fl.L[2][1] = slot[2 * 64];
        fl.rd[0] = slot[3 * 64];
        fl.rd[1] = slot[4 * 64];
        fl.rd[2] = slot[5 * 64];
        double Pm[M][M];
        Pm[0][0] = slot[6 * 64];
        Pm[0][1] = Pm[1][0] = slot[7 * 64];
        Pm[0][2] = Pm[2][0] = slot[8 * 64];
        Pm[1][1] = slot[9 * 64];
        Pm[1][2] = Pm[2][1] = slot[10 * 64];
        Pm[2][2] = slot[11 * 64];
        const double det = slot[12 * 64];
        double bf[M], q;
        collapsed_mean<M>(zc, yb.x, yb.y, f.R, f.rsig2, f.beta, Pm, fl, bf, q);
        if (fast) {
          if (!RECORD || det != 0.0) propagate_mean_f<M>(phi, f.p.delta, bf, f.beta);
          f.last_det = det;
          f.last_q = q;
          f.ld.mul(det);
          f.sumq += q;
          f.neg = f.neg || (det < 0.0);
        } else {
          const bool upd = det != 0.0;  // inv(F) threw: no update (filter.jl:151-154)
          if (upd) propagate_mean_f<M>(phi, f.p.delta, bf, f.beta);
          f.last_det = det;
          f.last_q = upd ? q : __builtin_nan("");
          if (t >= 1) {
            f.ld.mul(det);
            f.sumq += f.last_q;
            f.neg = f.neg || (det < 0.0);
          }
        }
      } else if (act) {
        // NaN column: prediction only; F, v stale → the loglik re-adds the previous term
        double bf[M];
#pragma unroll
        for (int i = 0; i < M; ++i) bf[i] = f.beta[i];
        propagate_mean_f<M>(phi, f.p.delta, bf, f.beta);
        if (t >= 1) {
          f.ld.mul(f.last_det);
          f.sumq += f.last_q;
          f.neg = f.neg || (f.last_det < 0.0);
        }
      }
      if constexpr (RECORD) {
        const int rs = t - max(0, my_steps - rec_len);
        if (live && !defer && act && rs >= 0) {
          const size_t o = (size_t)b * (size_t)rec_len + rs;
#pragma unroll
          for (int i = 0; i < M; ++i) rec_beta[o * M + i] = f.beta[i];
        }
      }
      if (tt == kSTB - 1) {
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();  // scratch reads done before the next block's writes
      }
    }
    end_iteration(k);
  }

  if (!live || defer) return;
  out[b] = f.loglik(nobs, flags);
  }

  };
  if (cov)
    role(std::true_type{});
  else
    role(std::false_type{});
}

namespace {

template <int NP>
hipError_t launch_split_np(const LaunchArgs& a) {
  const int interleave = 0;  // wave-to-role layout: covariance waves 0-3, mean waves 4-7 (1: alternating)
  const int grid = (a.B + kSplitPairs * 64 - 1) / (kSplitPairs * 64);
  if (a.rec_beta) {
    hipLaunchKernelGGL((dns_split_kernel<NP, true>), dim3(grid), dim3(kSplitBlock), 0, a.stream, a.theta, a.P, a.B,
                       a.space, a.panel, a.T, a.N, a.mats, a.T_use, a.out, a.flags, a.rec_beta, a.rec_P, a.horizon,
                       a.rec_len, a.defer_list, a.defer_count, interleave, a.flags_next);
  } else {
    hipLaunchKernelGGL((dns_split_kernel<NP, false>), dim3(grid), dim3(kSplitBlock), 0, a.stream, a.theta, a.P, a.B,
                       a.space, a.panel, a.T, a.N, a.mats, a.T_use, a.out, a.flags, nullptr, nullptr, 0, 0,
                       a.defer_list, a.defer_count, interleave, a.flags_next);
  }
  return hipGetLastError();
}

}  // namespace

bool dns_split_supported(int np) { return np == 8 || np == 16 || np == 24 || np == 30 || np == 32; }

hipError_t launch_dns_split(const LaunchArgs& a) {
  switch (a.np) {
    case 8: return launch_split_np<8>(a);
    case 16: return launch_split_np<16>(a);
    case 24: return launch_split_np<24>(a);
    case 30: return launch_split_np<30>(a);
    case 32: return launch_split_np<32>(a);
  }
  return hipErrorInvalidValue;
}

}  // namespace yfm

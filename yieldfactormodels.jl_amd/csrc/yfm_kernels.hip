// yfm_kernels.hip — batched Kalman log-likelihood kernels for gfx950 (MI355X).
//
// Hot path restated: get_loss (src/models/kalman/filter.jl:182-209) looping over
// filter! (filter.jl:125-179) from initialize_filter (filter.jl:1-10), evaluated for
// B parameter vectors at once (compute_loss, src/optimization.jl:10-23).
//
// Mapping: ONE FILTER PER LANE.  Every lane owns one candidate θ_b;
// its M×M state, the decoded parameters and its loadings Z (N×(M−1) non-constant
// columns) live in VGPRs.  All lanes walk the same time index t, so the panel
// column y_t is wave-uniform: the workgroup stages TC columns at a time into LDS
// (one coalesced global sweep per chunk, prefetched into registers one chunk ahead)
// and every lane reads them as LDS broadcasts.  Nothing N×N is ever formed.
//
// Per-step algebra — the COLLAPSED form: with G = Z'Z, R = σ²G⁻¹,
// ĉ_t = G⁻¹Z'y_t (cross-sectional OLS factors), r'r_t = ‖y_t − Zĉ_t‖²,
// c = ĉ_t − β and S = P + R (M×M, symmetric):
//     v'F⁻¹v = r'r/σ² + c'S⁻¹c,        log det F = (N−M) log σ² + log det G + log det S,
//     β_{t|t} = β + P S⁻¹ c,            P_{t|t}  = P S⁻¹ R,
// all exact rewrites of filter.jl:143-176 (F = ZPZ' + σ²I, K = PZ'F⁻¹, I − KZ).
// r'r is formed from CENTERED columns ỹ = y − ȳ1 (1 = Z e₁ for every candidate),
// which removes the y'y − ŷ'ŷ cancellation.  S is factorised by LDLᵀ.
// Lanes whose Z'Z is ill-conditioned (κ₁ ≥ 1e6), singular, or has fewer maturities than
// states (N < M) are appended to a deferral list and evaluated afterwards by the
// double-double CAPACITANCE kernel (yfm_fixedz_dd.hip): B̃ = σ²I + PG, pivoted LU,
// W = B̃⁻¹P, v'F⁻¹v = (v'v − u'Wu)/σ², P_{t|t} = σ²W, log det F = (N−M) log σ² +
// log det B̃.
//
// Panel layout in HBM (built by prep_panel_kernel from the caller's N×T
// column-major matrix): T columns of LDP = NP + 4 doubles —
//   [ ỹ_0 … ỹ_{N-1}, 0 … 0 (to NP), ȳ, ỹ'ỹ, isnan(any y), y'y ].
#include "yfm_fixedz.hpp"

namespace yfm {

constexpr int kBlock = 256;  // 4 waves: one per SIMD of a CU
constexpr int kTC = 64;  // panel columns per LDS chunk (DNS; GNS5 keeps 32: its z̃ scratch takes the LDS)
// Variants measured and not kept live in git history and DESIGN.md §3.1 / §6 (round 5 pruned them from the
// library): the look-ahead and pipelined steady blocks (the next block's MFMAs among the mean updates — FP64
// MFMA and VALU share one pipe on gfx950: 4.5% and 1.5% slower), four 8-byte z̃ stores per tile instead of
// the σ-permuted 16-byte ones, the first chunks loaded after the setup, no mid-block steady switch, MFMA A
// operands copied to VGPRs, two (4, 4) tile groups, chunk rotations after a block's steps, and the timing
// probes (phase cycle counters, MFMAs issued twice, z̃ never stored) that located the costs.
constexpr bool kMfma4 = true;   // GNS5 Z'ỹ on v_mfma_f64_4x4x4_4b_f64 (DNS keeps v_mfma_f64_16x16x4_f64)
constexpr bool kZBasis = true;  // GNS5 fragments e = 1 − e^{−λm} against (ỹ, ỹ/m): see the kernel

__global__ void prep_panel_kernel(const double* __restrict__ Y, int N, int T, int np, int ldp,
                                  double* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  const double* y = Y + (size_t)t * N;
  double* o = out + (size_t)t * ldp;
  double s1 = 0.0, yy = 0.0;
  bool nan = false;
  for (int i = 0; i < N; ++i) {
    const double v = y[i];
    nan = nan || (v != v);
    s1 += v;
    yy = fma(v, v, yy);
  }
  const double ybar = s1 / (double)N;
  double tt = 0.0;
  for (int i = 0; i < N; ++i) {
    const double d = y[i] - ybar;
    o[i] = d;
    tt = fma(d, d, tt);
  }
  for (int i = N; i < np; ++i) o[i] = 0.0;
  o[np] = ybar;
  o[np + 1] = tt;
  o[np + 2] = nan ? 1.0 : 0.0;
  o[np + 3] = yy;
}

// initialize_filter (filter.jl:1-10) for the 5-factor model in its own kernel: its 15×15
// Lyapunov solve needs ~480 VGPRs, which inside the filter kernel forced the whole filter to spill
// (≈2 KB per lane of scratch).  Writes β₀, the upper triangle of P₀ and the ok flag per candidate,
// structure-of-arrays (rec[q·B + b]) so the filter kernel's reads are coalesced.
template <int M>
constexpr int fz_rec_len() { return M + M * (M + 1) / 2 + 1; }

template <int M, int LEAD>
__global__ __launch_bounds__(256) void fixedz_init_kernel(const double* __restrict__ theta, int P, int B, int space,
                                                          double* __restrict__ rec, unsigned int* __restrict__ flags_next) {
  if (flags_next && blockIdx.x == 0 && threadIdx.x < kFlagsPerBank) flags_next[threadIdx.x] = 0u;  // the next launch's counters
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  Params<M, LEAD> p;
  decode_params<M, LEAD>(theta + (size_t)b * P, space, p);
  double beta[M], Pm[M][M];
  const bool ok = init_state<M, LEAD>(p, beta, Pm);
  int q = 0;
#pragma unroll
  for (int i = 0; i < M; ++i) rec[(size_t)(q++) * B + b] = beta[i];
#pragma unroll
  for (int i = 0; i < M; ++i)
#pragma unroll
    for (int j = i; j < M; ++j) rec[(size_t)(q++) * B + b] = Pm[i][j];
  rec[(size_t)q * B + b] = ok ? 1.0 : 0.0;
}

// The value of role O of this lane's aligned group of R lanes (R = 2: lane pairs, 4: quads): DPP quad_perm.
template <int R, int O>
__device__ __forceinline__ double role_bcast(double x) {
  static_assert(R == 2 || R == 4, "groups inside one quad");
  constexpr int ctrl = R == 4 ? (O | (O << 2) | (O << 4) | (O << 6)) : (O | (O << 2) | ((2 + O) << 4) | ((2 + O) << 6));
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), ctrl, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), ctrl, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
template <int R>
__device__ __forceinline__ double role_bcast_from(int o, double x) {  // o constant after unrolling
  if constexpr (R == 2) {
    return o == 0 ? role_bcast<2, 0>(x) : role_bcast<2, 1>(x);
  } else {
    return o == 0 ? role_bcast<4, 0>(x) : o == 1 ? role_bcast<4, 1>(x) : o == 2 ? role_bcast<4, 2>(x) : role_bcast<4, 3>(x);
  }
}

// fixedz_init_kernel with each candidate's Lyapunov system spread over R lanes (GNS5; launched with R = 2).  The per-lane kernel holds
// the augmented 15×16 system in 480 registers and spills 540 B/lane; here role o of a candidate's R lanes holds the
// columns c ≡ o (mod R) of [L | q] (16/R columns), so the system fits in registers.  The elimination is gauss_solve's
// arithmetic, operation for operation: per step every lane receives column k from its owner (DPP), runs the same
// pivot search on it (identical inputs → the same pivot in every role), exchanges rows k and p in its own columns
// and updates them with the same multipliers; back substitution runs gauss_solve's FMA chain in every lane with the
// entries of U broadcast from their owners.  The record is bitwise the per-lane kernel's.  Decoding and β₀ = (I − Φ)\δ
// are repeated in every role.
template <int M, int LEAD, int R>
__global__ __launch_bounds__(256) void fixedz_init_coop_kernel(const double* __restrict__ theta, int P, int B, int space,
                                                               double* __restrict__ rec,
                                                               unsigned int* __restrict__ flags_next) {
  if (flags_next && blockIdx.x == 0 && threadIdx.x < kFlagsPerBank) flags_next[threadIdx.x] = 0u;  // the next launch's counters
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = g / R;
  const int role = threadIdx.x & (R - 1);
  if (b >= B) return;  // B·R threads round up to whole groups: a group is live or not as a whole
  Params<M, LEAD> p;
  decode_params<M, LEAD>(theta + (size_t)b * P, space, p);
  double beta[M];
  bool ok;
  {
    double A[M][M], x[M][1];
#pragma unroll
    for (int i = 0; i < M; ++i) {
#pragma unroll
      for (int j = 0; j < M; ++j) A[i][j] = (i == j ? 1.0 : 0.0) - p.Phi[i][j];
      x[i][0] = p.delta[i];
    }
    ok = gauss_solve<M, 1>(A, x);
#pragma unroll
    for (int i = 0; i < M; ++i) beta[i] = x[i][0];
  }
  constexpr int S = M * (M + 1) / 2;     // unknowns P_kl, k ≤ l
  constexpr int NS = (S + 1 + R - 1) / R;  // local columns (the right-hand side is global column S)
  double a[NS][S];
  // build: row (i, j), column (k, l) of I − (the symmetric-subspace restriction of Φ⊗Φ), exactly init_state's;
  // column by column, each lane keeping its own (global column c → local column c / R of role c % R)
  {
    auto put = [&](int c, int r, double v) {
      if (c % R == 0) {
        a[c / R][r] = v;
      } else {
        a[c / R][r] = role == c % R ? v : a[c / R][r];
      }
    };
    int c = 0;
#pragma unroll
    for (int k = 0; k < M; ++k)
#pragma unroll
      for (int l = k; l < M; ++l, ++c) {
        int r = 0;
#pragma unroll
        for (int i = 0; i < M; ++i)
#pragma unroll
          for (int j = i; j < M; ++j, ++r) {
            double s = p.Phi[i][k] * p.Phi[j][l];
            if (k != l) s = fma(p.Phi[i][l], p.Phi[j][k], s);
            put(c, r, (r == c ? 1.0 : 0.0) - s);
          }
      }
    int r = 0;
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
      for (int j = i; j < M; ++j, ++r) {
        put(S, r, p.Q[i][j]);
#pragma unroll
        for (int c2 = S + 1; c2 < NS * R; ++c2) put(c2, r, 0.0);
      }
  }
  // elimination with partial pivoting (gauss_solve's pivot rule and arithmetic)
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const int o = k % R, sk = k / R;
    double col[S];
#pragma unroll
    for (int i = k; i < S; ++i) col[i] = role_bcast_from<R>(o, a[sk][i]);
    int pv = k;
    double amax = fabs(col[k]);
#pragma unroll
    for (int i = k + 1; i < S; ++i) {
      const double v = fabs(col[i]);
      const bool gt = v > amax;
      amax = gt ? v : amax;
      pv = gt ? i : pv;
    }
#pragma unroll
    for (int i = k + 1; i < S; ++i) {
      const bool sw = pv == i;
      const double ck = col[k], ci = col[i];
      col[k] = sw ? ci : ck;
      col[i] = sw ? ck : ci;
      // local columns below sk hold eliminated columns only; in slot sk the roles whose column is ≤ k exchange
      // and update entries below the diagonal that are never read again
#pragma unroll
      for (int s = sk; s < NS; ++s) {
        const double u = a[s][k], w = a[s][i];
        a[s][k] = sw ? w : u;
        a[s][i] = sw ? u : w;
      }
    }
    const double piv = col[k];
    ok = ok && (piv != 0.0);
    const double rp = 1.0 / piv;
#pragma unroll
    for (int i = k + 1; i < S; ++i) {
      const double l = col[i] * rp;
#pragma unroll
      for (int s = sk; s < NS; ++s) a[s][i] = fma(-l, a[s][k], a[s][i]);
    }
  }
  // back substitution: x_k = (q_k − Σ_{j>k} U_kj x_j) / U_kk in gauss_solve's order.  The running sum travels:
  // every lane applies its own column's entry and the result of the owner of column j is taken (x is replicated),
  // so no entry of U is copied out of its owner and each hop depends on the last
  double x[S];
#pragma unroll
  for (int k = S - 1; k >= 0; --k) {
    const double rp = role_bcast_from<R>(k % R, 1.0 / a[k / R][k]);
    double s = role_bcast_from<R>(S % R, a[S / R][k]);
#pragma unroll
    for (int j = k + 1; j < S; ++j) s = role_bcast_from<R>(j % R, fma(-a[j / R][k], x[j], s));
    x[k] = s * rp;
  }
  if (role != 0) return;
  int q = 0;
#pragma unroll
  for (int i = 0; i < M; ++i) rec[(size_t)(q++) * B + b] = beta[i];
#pragma unroll
  for (int r = 0; r < S; ++r) rec[(size_t)(q++) * B + b] = x[r];
  rec[(size_t)q * B + b] = ok ? 1.0 : 0.0;
}

// ---- per-step building blocks (all __forceinline__: the fast path is one basic block) ----

// z̃ = Z'ỹ_t for the NZ non-constant loading columns (Σỹ = 0 removes column 0).
template <int NP, int NZ>
__device__ __forceinline__ void dot_zt(const double* __restrict__ col, const double (&Zc)[NZ][NP], double (&zt)[NZ]) {
  double a[NZ][2];
#pragma unroll
  for (int cz = 0; cz < NZ; ++cz) {
    a[cz][0] = 0.0;
    a[cz][1] = 0.0;
  }
#pragma unroll
  for (int i = 0; i < NP; i += 2) {
    const double2 y2 = *reinterpret_cast<const double2*>(col + i);
#pragma unroll
    for (int cz = 0; cz < NZ; ++cz) {
      a[cz][0] = fma(Zc[cz][i], y2.x, a[cz][0]);
      a[cz][1] = fma(Zc[cz][i + 1], y2.y, a[cz][1]);
    }
  }
#pragma unroll
  for (int cz = 0; cz < NZ; ++cz) zt[cz] = a[cz][0] + a[cz][1];
}

typedef double yfm_double4 __attribute__((ext_vector_type(4)));

// Fixed-loading models: DNS (M = 3, one γ, dns.jl:51-65) and the 5-factor
// generalised NS extension (M = 5, two γ; SURVEY §8 a9, not in the reference).
// Z column 0 is ones; columns 1.. come in (slope, curvature) pairs per γ:
// S = (1 − e^{−λm})/(λm), C = S − e^{−λm}.
//
// Z'ỹ_t for a whole wave is a GEMM: [64 candidates × NZ loading columns] × [NP
// maturities] · [NP × 16 steps].  With MFMA (NZ = 2, DNS) each wave computes it for
// 16 steps at a time with v_mfma_f64_16x16x4_f64 — A = the wave's loadings (held in
// registers as MFMA fragments for the whole filter), B = the staged panel columns —
// and hands each lane its own (z̃₀, z̃₁) through a per-wave LDS scratch.  The VALU
// then runs only the M×M update.  Without MFMA (GNS5) the dot products are VALU FMAs
// computed one step ahead, inside the same basic block as the update.
// A wave-uniform fast path (no NaN column, every lane active, every lane collapsed,
// t ≥ 1) carries no per-lane masking; everything else takes the general path.
template <int NP, int M, int LEAD, bool RECORD, bool STEADY_ = false, bool SPLIT_FORM = false>
__global__ __launch_bounds__(kBlock, 1) void fixedz_loglik_kernel(
    const double* __restrict__ theta, int P, int B, int space, const double* __restrict__ panel, int T, int N,
    const double* __restrict__ mats, const int* __restrict__ T_use, double* __restrict__ out,
    unsigned int* __restrict__ flags, double* __restrict__ rec_beta, double* __restrict__ rec_P, int horizon,
    int rec_len, int* __restrict__ defer_list, int* __restrict__ defer_count, const double* __restrict__ init_rec,
    unsigned int* __restrict__ flags_next, int steady) {
  constexpr int LDP = NP + 4;
  // panel columns per LDS chunk: 64 for DNS (a chunk rotation, with its two block barriers, every 64 steps
  // instead of 32: 0.2040 → 0.2022 ms at config 2, profiles/r4/ab23/); 32 where the LDS is taken by GNS5's
  // z̃ scratch
  constexpr int TC = (M == 3) ? kTC : 32;
  constexpr bool USE_MFMA_ = (M - 1 == 2 || M - 1 == 4) && (NP <= 32);
  // frozen-covariance steady state (FixedZFilter): the loglik-mode DNS instantiation
  // with STEADY_ (the plain instantiation is the full recursion, YFM_DNS_STEADY=0)
  constexpr bool STEADY = STEADY_ && !RECORD && (M == 3 || M == 5) && USE_MFMA_;
  constexpr bool SPLIT_INIT = (M == 5);  // initial state from fixedz_init_kernel
  constexpr int CH = TC * LDP;               // doubles per chunk
  constexpr int PER = (CH + kBlock - 1) / kBlock;
  constexpr int NZ = M - 1;                   // non-constant loading columns
  constexpr bool USE_MFMA = (NZ == 2 || NZ == 4) && (NP <= 32);  // fragments + LDS scratch budget
  constexpr int NK = (NP + 3) / 4;            // MFMA k-steps (4 maturities each)
  constexpr int NRT = 64 * NZ / 16;           // MFMA row tiles per wave (16 (cand, col) pairs each)
  // row tiles accumulated at once (bounds live accumulators).  DNS: two groups of 4, so the first group's
  // z̃ stores overlap the second group's MFMAs (8: 0.2173 → 4: 0.2165 ms at config 2, 2: 0.2197 ms — two
  // accumulator chains expose the MFMA latency; profiles/r4/ab9, ab10)
  constexpr int RGN = 4;
  constexpr int RGN4 = (NZ == 2) ? NRT : 8;   // the same for the 4×4×4 form (one double per accumulator)
  constexpr int TB = 16;                      // steps per MFMA block
  // GNS5 (two γ): the MFMA rows are e_l = 1 − e^{−λ_l m} (one per γ) against the panel columns ỹ and
  // ỹ/m, so a candidate holds LEAD fragment rows instead of NZ = 2·LEAD:
  //   Σ S_l ỹ = (1/λ_l) Σ e_l ỹ/m,   Σ C_l ỹ = Σ (S_l − z_l) ỹ = Σ S_l ỹ + Σ e_l ỹ   (Σ ỹ = 0),
  // which halves the fragment registers (the 5-state filter no longer spills).
  constexpr bool ZB = USE_MFMA && kMfma4 && kZBasis && LEAD == 2;
  constexpr int RPC = ZB ? LEAD : NZ;         // fragment rows per candidate
  constexpr int NRTA = 64 * RPC / 16;         // fragment row tiles per wave
  constexpr int SS = 64 * NZ + 2;             // scratch row stride (doubles): one row per step
  // (also the fragment staging image of 32 candidates: 32·RPC rows of 4·NK + 1 maturities)
  constexpr int SCR = USE_MFMA ? ((TB * SS > 32 * RPC * (4 * NK + 1)) ? TB * SS : 32 * RPC * (4 * NK + 1)) : 2;
  static_assert(NZ == 2 * LEAD, "loading columns come in (S, C) pairs per gamma");
  static_assert(NP % 2 == 0, "double2 panel reads");
  static_assert(TC % TB == 0, "MFMA blocks tile the panel chunk");
  __shared__ __attribute__((aligned(16))) double sh[2][CH];
  __shared__ __attribute__((aligned(16))) double scratch[kBlock / 64][SCR];
  __shared__ int s_nobs_max;
  __shared__ double s_rm[ZB ? NP : 1];  // 1/m_i (0 past N)

  if (flags_next && blockIdx.x == 0 && threadIdx.x < kFlagsPerBank) flags_next[threadIdx.x] = 0u;  // the next launch's counters
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int b = blockIdx.x * kBlock + tid;
  const bool live = b < B;
  const int bb = live ? b : (B - 1);
  const int nobs = T_use ? T_use[bb] : T;

  // panel chunk loads (PER doubles per thread; LDS holds chunks c and c+1 while chunk c is processed)
  auto load_into = [&](double* dst, int c) {
    const size_t base = (size_t)c * CH;
    const size_t lim = (size_t)T * LDP;
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      const int e = r * kBlock + tid;
      const size_t g = base + e;
      dst[r] = (e < CH && g < lim) ? panel[g] : 0.0;
    }
  };
  auto store_from = [&](const double* src, double* buf) {
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      const int e = r * kBlock + tid;
      if (e < CH) buf[e] = src[r];
    }
  };
  // EARLY: chunks 0 and 1 issued before the setup, so their HBM latency hides under the θ decode and the
  // loadings instead of two serial round trips after it (stored to LDS where the staging starts below)
  constexpr bool EARLY = M == 3 && NP <= 32;  // GNS5 and NP > 32 spill with the 2·PER registers
  double pre0[EARLY ? PER : 1], pre1[EARLY ? PER : 1];
  if constexpr (EARLY) {
    load_into(pre0, 0);
    load_into(pre1, 1);
  }

  if (tid == 0) s_nobs_max = 0;
  if constexpr (ZB) {
    for (int i = tid; i < NP; i += kBlock) s_rm[i] = (i < N) ? 1.0 / mats[i] : 0.0;
  }
  __syncthreads();
  // loglik mode (horizon = 0): filter! over columns 0 .. nobs−2 (filter.jl:190).  Trajectory
  // mode (horizon ≥ 1, predict, filter.jl:250-282): columns 0 .. nobs−1, then horizon NaN
  // steps (the NaN padding of forecasting.jl:141 plus predict's final NaN step).
  const int my_steps = horizon > 0 ? nobs + horizon : nobs - 1;
  const int my_data = horizon > 0 ? nobs : nobs - 1;  // steps t < my_data read column t
  atomicMax(&s_nobs_max, live ? my_steps : 0);

  // ---- decode θ_b, loadings, Z'Z, initial state ----------------------------------
  // The wave's 64 θ rows are contiguous (64·P doubles): staged through the wave's scratch with coalesced
  // loads (a lane reading its own row directly touches one cache line per lane and parameter), then each
  // lane decodes its row from LDS.  Needs the model's own parameter count and room in the scratch.
  constexpr int kP = param_count(M, LEAD);
  const double* th_row = theta + (size_t)bb * P;
  if constexpr (USE_MFMA && 64 * kP <= SCR) {
    if (P == kP) {
      const int w0 = min(blockIdx.x * kBlock + wave * 64, B - 1);  // first row of this wave's range
      const int n = min(64, B - w0) * kP;
      const double* src = theta + (size_t)w0 * kP;
      double* thl = scratch[wave];
      double v[kP];
#pragma unroll
      for (int r = 0; r < kP; ++r) {
        const int e = r * 64 + lane;
        v[r] = (e < n) ? src[e] : 0.0;
      }
#pragma unroll
      for (int r = 0; r < kP; ++r) thl[r * 64 + lane] = v[r];
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own rows
      __builtin_amdgcn_wave_barrier();
      th_row = thl + (bb - w0) * kP;
    }
  }
  Params<M, LEAD> p;
  decode_params<M, LEAD>(th_row, space, p);
  __builtin_amdgcn_s_waitcnt(0xc07f);  // the rows are read before the fragment staging reuses the scratch
  __builtin_amdgcn_wave_barrier();

  double Zc[NZ][NP];
#pragma unroll
  for (int l = 0; l < LEAD; ++l) {
    const double lam = 1e-2 + exp(p.gam[l]);  // dns.jl:55
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      // branch-free (maturities past N computed on a clamped index and zeroed): with `if (i < N)` every
      // maturity was its own basic block and the 30 exp/div chains ran one after another
      const double tau = lam * mats[max(min(i, N - 1), 0)];
      const double z = exp(-tau);
      const double s = (1.0 - z) / tau;
      Zc[2 * l][i] = (i < N) ? s : 0.0;
      Zc[2 * l + 1][i] = (i < N) ? s - z : 0.0;
    }
  }
  double G[M][M];
  G[0][0] = (double)N;
#pragma unroll
  for (int c = 0; c < NZ; ++c) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NP; ++i) s += Zc[c][i];
    G[0][c + 1] = s;
    G[c + 1][0] = s;
#pragma unroll
    for (int d = c; d < NZ; ++d) {
      double g = 0.0;
#pragma unroll
      for (int i = 0; i < NP; ++i) g = fma(Zc[c][i], Zc[d][i], g);
      G[c + 1][d + 1] = g;
      G[d + 1][c + 1] = g;
    }
  }

  // MFMA A fragments: tile r, k-step kk — lane l holds Z of pair p = 16r + σ(l & 15)
  // (candidate p / NZ of this wave, column p % NZ) at maturity 4kk + (l >> 4).
  // Gathered once through the wave's scratch, 16 candidates at a time.
  // σ (the 16×16×4 form only): row i = g + 4q of a tile holds pair 16r + 4g + q, so the four D values a lane
  // holds (rows g, g+4, g+8, g+12 of one step) are four consecutive pairs — two 16-byte LDS stores per tile
  // instead of four 8-byte ones, and still one candidate's z̃ in consecutive doubles for the step reads
  constexpr bool SIGMA = USE_MFMA && !ZB && !(kMfma4 && NZ == 4);
  // IL: the row tiles in three groups (4, 2, 2), each group's stores interleaved with the next group's MFMAs
  // (NP 29–32: one store per k-step)
  constexpr bool IL = SIGMA && NRT == 2 * RGN && NK == 2 * RGN;
  constexpr bool IL5 = ZB && NK == NRTA;  // GNS5: the same across step pairs
  auto sigma = [](int i) { return SIGMA ? 4 * (i & 3) + (i >> 2) : i; };
  double Af[USE_MFMA ? NRTA : 1][USE_MFMA ? NK : 1];
  double rlam[LEAD];  // 1/λ_l (z-basis fragments)
#pragma unroll
  for (int l = 0; l < LEAD; ++l) rlam[l] = 1.0 / (1e-2 + exp(p.gam[l]));
  if constexpr (USE_MFMA) {
    constexpr int ZS = 4 * NK + 1;  // maturity stride of the staging image (odd: conflict-free LDS)
    constexpr int HT = NRTA / 2;    // row tiles per half wave (32 candidates)
    static_assert(32 * RPC * ZS <= SCR, "staging fits the scratch");
    // two rounds of 32 candidates (round 3: four of 16, with a block barrier after each write and read — the
    // scratch is the wave's own, so the wave's LDS counter and a wave barrier order it; profiles/r4/ab13)
    double* st = scratch[wave];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if ((lane >> 5) == h) {
        const int cl = lane & 31;
        if constexpr (ZB) {
#pragma unroll
          for (int l = 0; l < LEAD; ++l) {
            const double lam = 1e-2 + exp(p.gam[l]);
#pragma unroll
            for (int m = 0; m < ZS; ++m) {
              const double e = 1.0 - exp(-(lam * mats[max(min(m, N - 1), 0)]));
              st[(cl * RPC + l) * ZS + m] = (m < N) ? e : 0.0;
            }
          }
        } else {
#pragma unroll
          for (int c = 0; c < NZ; ++c)
#pragma unroll
            for (int m = 0; m < ZS; ++m) st[(cl * NZ + c) * ZS + m] = (m < NP) ? Zc[c][m] : 0.0;
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int r = h * HT; r < (h + 1) * HT; ++r) {
        const int pr = 16 * r + sigma(lane & 15) - h * 32 * RPC;  // pair index within this half
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) Af[r][kk] = st[pr * ZS + 4 * kk + (lane >> 4)];
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
  }

  FixedZFilter<M, LEAD, RECORD, STEADY, SPLIT_FORM> f;
  f.p = p;
  f.steady_ok = steady != 0;
  f.setup(G, N, !SPLIT_INIT);
  if constexpr (SPLIT_INIT) {
    int q = 0;
#pragma unroll
    for (int i = 0; i < M; ++i) f.beta[i] = init_rec[(size_t)(q++) * B + bb];
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
      for (int j = i; j < M; ++j) {
        const double v = init_rec[(size_t)(q++) * B + bb];
        f.Pm[i][j] = v;
        f.Pm[j][i] = v;
      }
    f.init_ok = init_rec[(size_t)q * B + bb] != 0.0;
  }
  // ill-conditioned Z'Z: this candidate is evaluated by the double-double capacitance kernel
  // instead (yfm_fixedz_dd.hip); its lane here runs along without writing
  const bool defer = live && !f.collapsed;
  if (defer) defer_list[atomicAdd(defer_count, 1)] = b;

  // wave-uniform facts for the fast path
  int wmin = live ? my_data : 0x7fffffff;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) wmin = min(wmin, __shfl_xor(wmin, off));
  const int wave_min_data = __builtin_amdgcn_readfirstlane(wmin);
  const bool wave_all_collapsed = true;  // non-collapsed lanes are deferred (their values are discarded)

  __syncthreads();
  const int nsteps = max(s_nobs_max, 0);

  // ---- panel staging: LDS holds chunks c and c+1 while chunk c is processed ----------
  double pre[PER];
  auto load_chunk = [&](int c) { load_into(pre, c); };
  auto store_chunk = [&](double* buf) { store_from(pre, buf); };
  if (nsteps > 0) {
    if constexpr (EARLY) {
      store_from(pre0, sh[0]);
      store_from(pre1, sh[1]);
    } else {
      load_chunk(0);
      store_chunk(sh[0]);
      load_chunk(1);
      store_chunk(sh[1]);
    }
    __syncthreads();
    load_chunk(2);
  }
  auto col_of = [&](int t) -> const double* { return sh[(t / TC) & 1] + (t % TC) * LDP; };
  // a 16×16×4 D tile into a scratch buffer: lane l holds step l & 15, pairs 16r + 4(l >> 4) + q (σ above)
  auto store_tile = [&](double* dst, int r, const yfm_double4& a) {
    if constexpr (SIGMA) {
      double* d = dst + (lane & 15) * SS + 16 * r + 4 * (lane >> 4);
      *reinterpret_cast<double2*>(d) = make_double2(a[0], a[1]);
      *reinterpret_cast<double2*>(d + 2) = make_double2(a[2], a[3]);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) dst[(lane & 15) * SS + 16 * r + (lane >> 4) + 4 * q] = a[q];
    }
  };

  // one filter step given z̃_t (zc), (ȳ, ỹ'ỹ) and (nanflag, y'y) of column t
  auto do_step = [&](int t, const double (&zc)[NZ], double2 yb_c, double2 meta_c) {
    const bool fast = (t >= 1) && (meta_c.x == 0.0) && (t < wave_min_data) && wave_all_collapsed;
    f.step(t, zc, yb_c, meta_c, fast, my_steps, my_data);
  };
  auto record = [&](int t) {
    if constexpr (RECORD) {
      if (live && !defer) f.record(t, b, my_steps, rec_len, rec_beta, rec_P);
    }
  };
  auto rotate = [&](int t) {  // after step t: if chunk c = t / TC is done, its buffer takes chunk c + 2
    if ((t + 1) % TC == 0) {
      const int c = t / TC;
      __syncthreads();
      store_chunk(sh[c & 1]);
      __syncthreads();
      load_chunk(c + 3);
    }
  };

  if constexpr (USE_MFMA) {
    unsigned int steady_steps = 0;  // STEADY: this wave's steady steps (one atomic at the end: a per-block
                                    // atomic would put its latency on the next global load's wait)
    // a block-end chunk rotation, deferred to the next block's start: with its barrier after the steps the
    // compiler sinks the steps' arithmetic below it and issues all 32 operand reads up front (128 registers)
    int rot_t = -1;
    for (int t0 = 0; t0 < nsteps; t0 += TB) {
      if (rot_t >= 0) {
        rotate(rot_t);
        rot_t = -1;
      }
      // the freeze rule's contraction bound, once per lane, at a block boundary before the block's MFMA
      // accumulators are live (FixedZFilter::prepare_bound)
      if constexpr (STEADY) f.prepare_bound();
      if constexpr (SIGMA || M == 5) {
        // the A fragments stay in AGPRs, where the 16×16×4 MFMA reads them as its A operand (left to itself the
        // allocator copies each one to a VGPR before its MFMA: 128 v_accvgpr_read per block)
#pragma unroll
        for (int r = 0; r < NRTA; ++r)
#pragma unroll
          for (int kk = 0; kk < NK; ++kk) asm volatile("" : "+a"(Af[r][kk]));
      }
      double* scr = scratch[wave];
      // ---- z̃ for steps t0 .. t0+15 of all 64 candidates: NRT·NK MFMAs ----
      const double* cb = col_of(t0);  // TB consecutive columns of one chunk
      // the block's NaN flags, one column per lane, read before the MFMAs so the steady-block vote after them
      // does not wait for an LDS round trip (0.2179 → 0.2168 ms at config 2, profiles/r4/ab9/)
      const double col_flag = cb[min(lane, TB - 1) * LDP + NP + 2];
      if constexpr (ZB && IL5) {
        // as below, software-pipelined over the step pairs: step pair sp − 1's 8 results are stored one per
        // k-step of step pair sp's MFMAs (the wave issues the stores while the matrix pipe works)
        double accp[NRTA];
#pragma unroll
        for (int sp = 0; sp <= TB / 2; ++sp) {
          double acc[NRTA];
          if (sp < TB / 2) {
            double bv[NK];
#pragma unroll
            for (int kk = 0; kk < NK; ++kk) {
              const int m = 4 * kk + (lane >> 4);
              const double y = (m < NP) ? cb[(2 * sp + ((lane & 3) >> 1)) * LDP + m] : 0.0;
              bv[kk] = (lane & 1) ? y * s_rm[m < NP ? m : 0] : y;
            }
#pragma unroll
            for (int r = 0; r < NRTA; ++r) acc[r] = 0.0;
#pragma unroll
            for (int kk = 0; kk < NK; ++kk) {
#pragma unroll
              for (int r = 0; r < NRTA; ++r)
                acc[r] = __builtin_amdgcn_mfma_f64_4x4x4f64(Af[r][kk], bv[kk], acc[r], 0, 0, 0);
              if (sp > 0)
                scr[(2 * (sp - 1) + ((lane & 3) >> 1)) * SS + 2 * (16 * kk + 4 * ((lane >> 2) & 3) + (lane >> 4)) +
                    (lane & 1)] = accp[kk];
            }
          } else {
#pragma unroll
            for (int r = 0; r < NRTA; ++r)
              scr[(2 * (sp - 1) + ((lane & 3) >> 1)) * SS + 2 * (16 * r + 4 * ((lane >> 2) & 3) + (lane >> 4)) +
                  (lane & 1)] = accp[r];
          }
          if (sp < TB / 2) {
#pragma unroll
            for (int r = 0; r < NRTA; ++r) accp[r] = acc[r];
          }
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NRTA * NK, 0);  // step pair 0's MFMAs
#pragma unroll
        for (int sp = 1; sp < TB / 2; ++sp)
#pragma unroll
          for (int kk = 0; kk < NK; ++kk) {
            __builtin_amdgcn_sched_group_barrier(0x008, NRTA, 0);  // a k-step of step pair sp
            __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);     // one store of step pair sp − 1
          }
      } else if constexpr (ZB) {
        // rows: pair 16r + 4blk + i = (candidate, γ index); columns j of step pair sp: step
        // 2sp + (j >> 1), ỹ (j even) or ỹ/m (j odd)
#pragma unroll
        for (int sp = 0; sp < TB / 2; ++sp) {
          double bv[NK];
#pragma unroll
          for (int kk = 0; kk < NK; ++kk) {
            const int m = 4 * kk + (lane >> 4);
            const double y = (m < NP) ? cb[(2 * sp + ((lane & 3) >> 1)) * LDP + m] : 0.0;
            bv[kk] = (lane & 1) ? y * s_rm[m < NP ? m : 0] : y;
          }
#pragma unroll
          for (int r0 = 0; r0 < NRTA; r0 += NRTA) {
            double acc[NRTA];
#pragma unroll
            for (int r = 0; r < NRTA; ++r) acc[r] = 0.0;
#pragma unroll
            for (int kk = 0; kk < NK; ++kk)
#pragma unroll
              for (int r = 0; r < NRTA; ++r)
                acc[r] = __builtin_amdgcn_mfma_f64_4x4x4f64(Af[r][kk], bv[kk], acc[r], 0, 0, 0);
            // lane l: pair 16r + 4((l >> 2) & 3) + (l >> 4), step 2sp + ((l & 3) >> 1), column l & 1;
            // per step a candidate's four values are (Σe₁ỹ, Σe₁ỹ/m, Σe₂ỹ, Σe₂ỹ/m)
#pragma unroll
            for (int r = 0; r < NRTA; ++r)
              scr[(2 * sp + ((lane & 3) >> 1)) * SS + 2 * (16 * r + 4 * ((lane >> 2) & 3) + (lane >> 4)) + (lane & 1)] =
                  acc[r];
          }
        }
      } else if constexpr (kMfma4 && NZ == 4) {
        // v_mfma_f64_4x4x4_4b_f64: block blk of instruction (r, s, kk) is D[4×4] = A[4 pairs ×
        // 4 maturities]·B[4 maturities × 4 steps] for pairs 16r + 4blk + i, steps 4s + j,
        // maturities 4kk + k.  Operand lanes (tools/mfma_f64_4x4_probe.hip): A[blk][i][k] in
        // lane 16k + 4blk + i — exactly the 16×16×4 A fragment above — B[blk][k][j] in lane
        // 16k + 4blk + j (the same panel values for every block), D[blk][i][j] in lane
        // 16i + 4blk + j.  512 flops per instruction at ≈17 cycles vs 2,048 at ≈144 for the
        // 16×16×4 form at one wave per SIMD (profiles/r2/micro).
#pragma unroll
        for (int s = 0; s < TB / 4; ++s) {
          double bv[NK];
#pragma unroll
          for (int kk = 0; kk < NK; ++kk) {
            const int m = 4 * kk + (lane >> 4);
            bv[kk] = (m < NP) ? cb[(4 * s + (lane & 3)) * LDP + m] : 0.0;
          }
#pragma unroll
          for (int r0 = 0; r0 < NRT; r0 += RGN4) {
            double acc[RGN4];
#pragma unroll
            for (int r = 0; r < RGN4; ++r) acc[r] = 0.0;
#pragma unroll
            for (int kk = 0; kk < NK; ++kk)
#pragma unroll
              for (int r = 0; r < RGN4; ++r)
                acc[r] = __builtin_amdgcn_mfma_f64_4x4x4f64(Af[r0 + r][kk], bv[kk], acc[r], 0, 0, 0);
            // lane l holds pair 16r + 4((l >> 2) & 3) + (l >> 4) at step 4s + (l & 3)
#pragma unroll
            for (int r = 0; r < RGN4; ++r)
              scr[(4 * s + (lane & 3)) * SS + 16 * (r0 + r) + 4 * ((lane >> 2) & 3) + (lane >> 4)] = acc[r];
          }
        }
      } else {
        double bvk[NK];
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
          const int m = 4 * kk + (lane >> 4);
          bvk[kk] = (m < NP) ? cb[(lane & 15) * LDP + m] : 0.0;  // B[k = m][col = step]
        }
        if constexpr (IL) {
          // three groups of 4, 2, 2 tiles: the first group's 8 stores during the second group's MFMAs, the
          // second's 4 during the third's, so only the last 2 tiles' 4 stores trail the block
          constexpr int H = RGN / 2;
          yfm_double4 a1[RGN], a2[H], a3[H];
#pragma unroll
          for (int r = 0; r < RGN; ++r) a1[r] = yfm_double4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int r = 0; r < H; ++r) a2[r] = a3[r] = yfm_double4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int kk = 0; kk < NK; ++kk)
#pragma unroll
            for (int r = 0; r < RGN; ++r)
              a1[r] = __builtin_amdgcn_mfma_f64_16x16x4f64(Af[r][kk], bvk[kk], a1[r], 0, 0, 0);
#pragma unroll
          for (int kk = 0; kk < NK; ++kk) {
#pragma unroll
            for (int r = 0; r < H; ++r)
              a2[r] = __builtin_amdgcn_mfma_f64_16x16x4f64(Af[RGN + r][kk], bvk[kk], a2[r], 0, 0, 0);
            const int r1 = kk >> 1, h = kk & 1;
            double* d = scr + (lane & 15) * SS + 16 * r1 + 4 * (lane >> 4) + 2 * h;
            *reinterpret_cast<double2*>(d) = make_double2(a1[r1][2 * h], a1[r1][2 * h + 1]);
          }
#pragma unroll
          for (int kk = 0; kk < NK; ++kk) {
#pragma unroll
            for (int r = 0; r < H; ++r)
              a3[r] = __builtin_amdgcn_mfma_f64_16x16x4f64(Af[RGN + H + r][kk], bvk[kk], a3[r], 0, 0, 0);
            if (kk & 1) {
              const int r2 = kk >> 2, h = (kk >> 1) & 1;
              double* d = scr + (lane & 15) * SS + 16 * (RGN + r2) + 4 * (lane >> 4) + 2 * h;
              *reinterpret_cast<double2*>(d) = make_double2(a2[r2][2 * h], a2[r2][2 * h + 1]);
            }
          }
          __builtin_amdgcn_sched_group_barrier(0x008, RGN * NK, 0);  // the first group's MFMAs
#pragma unroll
          for (int kk = 0; kk < NK; ++kk) {
            __builtin_amdgcn_sched_group_barrier(0x008, H, 0);  // a k-step of the second group
            __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // one store of the first
          }
#pragma unroll
          for (int kk = 0; kk < NK; ++kk) {
            __builtin_amdgcn_sched_group_barrier(0x008, H, 0);  // a k-step of the third group
            if (kk & 1) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // one store of the second
          }
#pragma unroll
          for (int r = 0; r < H; ++r) store_tile(scr, RGN + H + r, a3[r]);
        } else {
#pragma unroll
        for (int r0 = 0; r0 < NRT; r0 += RGN) {
          yfm_double4 acc[RGN];
#pragma unroll
          for (int r = 0; r < RGN; ++r) acc[r] = yfm_double4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int kk = 0; kk < NK; ++kk)
#pragma unroll
            for (int r = 0; r < RGN; ++r)
              acc[r] = __builtin_amdgcn_mfma_f64_16x16x4f64(Af[r0 + r][kk], bvk[kk], acc[r], 0, 0, 0);
          // D[row][col = step]: lane l holds step l & 15, rows (l >> 4) + 4q = pairs 16r + 4(l >> 4) + q
#pragma unroll
          for (int r = 0; r < RGN; ++r) store_tile(scr, r0 + r, acc[r]);
        }
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's scratch writes landed
      __builtin_amdgcn_wave_barrier();
      const int tend = min(TB, nsteps - t0);
      // a block of steady steps: every lane of the wave frozen, and every step of the block a data
      // step of every lane (no NaN column, t ≥ 1, inside every lane's window)
      bool blk_steady = false;
      if constexpr (STEADY) {
        // (wave_frozen is wave-uniform here — wave_freeze re-establishes it after every full block; the
        // vote keeps the branch uniform even so)
        if (__all(f.wave_frozen) && t0 >= 1 && t0 + tend <= wave_min_data) {
          // the block's NaN flags, one column per lane: one LDS round trip instead of tend serial ones
          // (0.236 → 0.217 ms at config 2, profiles/r3/probes/dns_steady_nan/)
          const bool col_nan = (lane < tend) && (col_flag != 0.0);
          blk_steady = !__any(col_nan);
        }
      }
      // step operands for tt are read one step ahead (hides the LDS latency at 1 wave/SIMD)
      auto read_z = [&](int tt, double (&z)[NZ]) {  // this lane's pairs NZ·lane .. NZ·lane + NZ − 1
        const double* sp = scr + tt * SS + NZ * lane;
#pragma unroll
        for (int j = 0; j < NZ; j += 2) {
          const double2 v = *reinterpret_cast<const double2*>(sp + j);
          if constexpr (ZB) {
            z[j] = rlam[j / 2] * v.y;  // Σ S ỹ
            z[j + 1] = z[j] + v.x;     // Σ C ỹ
          } else {
            z[j] = v.x;
            z[j + 1] = v.y;
          }
        }
      };
      double zc[NZ];
      read_z(0, zc);
      double2 yb = *reinterpret_cast<const double2*>(cb + NP);
      double2 meta = *reinterpret_cast<const double2*>(cb + NP + 2);
      // two steps per trip with the operand buffers swapped by name (no register copies)
      double zn[NZ];
      double2 ybn, metan;
      auto half = [&](int tt, const double (&zc_)[NZ], double2 yb_, double2 meta_, double (&zn_)[NZ], double2& ybn_,
                      double2& metan_) {
        const int t = t0 + tt;
        const int tn = min(tt + 1, TB - 1);
        read_z(tn, zn_);
        ybn_ = *reinterpret_cast<const double2*>(cb + tn * LDP + NP);
        metan_ = *reinterpret_cast<const double2*>(cb + tn * LDP + NP + 2);
        do_step(t, zc_, yb_, meta_);
        record(t);
        if ((t + 1) % TC == 0) rot_t = t;  // the chunk rotation, deferred to the next block's start
      };
      // the mean update only, with the cached factors of S (bitwise the full step's values for a frozen lane);
      // operands read one step ahead as in `half`
      auto shalf = [&](int tt, const double (&zc_)[NZ], double2 yb_, double (&zn_)[NZ], double2& ybn_) {
        const int tn = min(tt + 1, TB - 1);
        read_z(tn, zn_);
        ybn_ = *reinterpret_cast<const double2*>(cb + tn * LDP + NP);
        f.steady_step(zc_, yb_);
        if ((t0 + tt + 1) % TC == 0) rot_t = t0 + tt;
      };
      if constexpr (STEADY) {
        if (blk_steady) {
          if (tend == TB) {
            // a whole block: the 16 steps unrolled into one basic block (no loop control or operand copies;
            // the chunk rotation, which only the block's last step can trigger, after it): 0.2114 → 0.2042 ms
            // at config 2, bitwise the same logliks (profiles/r4/ab16/)
            double zq[2][NZ];
            double2 ybq[2];
#pragma unroll
            for (int j = 0; j < NZ; ++j) zq[0][j] = zc[j];
            ybq[0] = yb;
#pragma unroll
            for (int u = 0; u < TB; ++u) {
              const int cur = u & 1, nx = cur ^ 1;
              const int tn = min(u + 1, TB - 1);
              read_z(tn, zq[nx]);
              ybq[nx] = *reinterpret_cast<const double2*>(cb + tn * LDP + NP);
              f.steady_step(zq[cur], ybq[cur]);
            }
            rot_t = ((t0 + TB) % TC == 0) ? t0 + TB - 1 : -1;  // at the next block's start
          } else {
            int tt = 0;
            for (; tt + 1 < tend; tt += 2) {
              shalf(tt, zc, yb, zn, ybn);
              shalf(tt + 1, zn, ybn, zc, yb);
            }
            if (tt < tend) shalf(tt, zc, yb, zn, ybn);
          }
          steady_steps += tend;
          f.count_steady(tend);
        }
      }
      if (!blk_steady) {
        int tt = 0;
        bool rest_steady = false;  // the rest of this block runs in the steady loop
        for (; tt + 1 < tend; tt += 2) {
          half(tt, zc, yb, meta, zn, ybn, metan);
          half(tt + 1, zn, ybn, metan, zc, yb, meta);
          if constexpr (STEADY) {
            // mid-block as well: lanes may freeze within this block (without it the config-2 steady share
            // drops 0.973 → 0.947, 0.226 → 0.234 ms; profiles/r4/exp1/)
            if (tt == TB / 2 - 2) f.prepare_bound();
            {
              // from the block's second half on, at every step pair: once every lane is frozen (the wave
              // vote of the block's end, taken early) and the rest of the block is data steps of every lane
              // with no NaN column, the remaining steps run as steady steps — the first block's waves freeze
              // at steps 10–14 (tools/steady_rule.py), so up to 6 of its 16 full steps become steady ones.
              // The lanes' values are bitwise the same either way (the steady step is the full step of a
              // frozen lane); only which loop runs them changes
              const int r0 = tt + 2;
              if (r0 >= TB / 2 && r0 < tend && t0 + tend <= wave_min_data) {
                const bool nan_rest = (lane >= r0) && (lane < tend) && (col_flag != 0.0);
                if (!__any(nan_rest)) {
                  f.wave_freeze(live && !defer && f.init_ok && t0 + tend <= my_steps);
                  if (f.wave_frozen) {  // wave-uniform (wave_freeze votes)
                    rest_steady = true;
                    tt = r0;
                    break;
                  }
                }
              }
            }
          }
        }
        if constexpr (STEADY) {
          if (rest_steady) {  // step tt's operands are in (zc, yb): read ahead by the last `half`
            const int n = tend - tt;
            for (; tt + 1 < tend; tt += 2) {
              shalf(tt, zc, yb, zn, ybn);
              shalf(tt + 1, zn, ybn, zc, yb);
            }
            if (tt < tend) shalf(tt, zc, yb, zn, ybn);
            steady_steps += n;
            f.count_steady(n);
          }
        }
        if (!rest_steady) {
          if (tt < tend) half(tt, zc, yb, meta, zn, ybn, metan);
          if constexpr (STEADY) f.wave_freeze(live && !defer && f.init_ok && t0 + tend <= my_steps);
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();  // scratch reads done before the next block's writes
    }
    if (rot_t >= 0) rotate(rot_t);  // every wave passes the same barriers
    if constexpr (STEADY) {
      if (lane == 0 && steady_steps) atomicAdd(&flags[4], steady_steps);  // yfm_last_batch_steady
    }
  } else {
    double zc[NZ];
    double2 yb_c = make_double2(0.0, 0.0), meta_c = make_double2(0.0, 0.0);
    if (nsteps > 0) {
      const double* c0 = col_of(0);
      dot_zt<NP, NZ>(c0, Zc, zc);
      yb_c = *reinterpret_cast<const double2*>(c0 + NP);
      meta_c = *reinterpret_cast<const double2*>(c0 + NP + 2);
    }
    // two steps per trip with the operand buffers swapped by name (as in the MFMA path)
    double zn[NZ];
    double2 yb_n, meta_n;
    auto half = [&](int t, const double (&zc_)[NZ], double2 yb_, double2 meta_, double (&zn_)[NZ], double2& ybn_,
                    double2& metan_) {
      const double* cn = col_of(t + 1);  // t + 1 ≤ nsteps ≤ T − 1: a resident panel column
      dot_zt<NP, NZ>(cn, Zc, zn_);
      ybn_ = *reinterpret_cast<const double2*>(cn + NP);
      metan_ = *reinterpret_cast<const double2*>(cn + NP + 2);
      do_step(t, zc_, yb_, meta_);
      record(t);
      rotate(t);
    };
    int t = 0;
    for (; t + 1 < nsteps; t += 2) {
      half(t, zc, yb_c, meta_c, zn, yb_n, meta_n);
      half(t + 1, zn, yb_n, meta_n, zc, yb_c, meta_c);
    }
    if (t < nsteps) half(t, zc, yb_c, meta_c, zn, yb_n, meta_n);
  }

  if (!live || defer) return;
  const double ll = f.loglik(nobs, flags);
  out[b] = ll;
}

}  // namespace yfm

// ------------------------------------------------------------------------------------
// host-side dispatch (declared in yfm_internal.hpp)
// ------------------------------------------------------------------------------------
#include "yfm_internal.hpp"

#include <cstdlib>

namespace yfm {

// the frozen-covariance steady state of the DNS loglik kernel (FixedZFilter): on unless YFM_DNS_STEADY=0
static int steady_enabled() {
  const char* e = std::getenv("YFM_DNS_STEADY");
  return (e && e[0] == '0') ? 0 : 1;
}

// the GNS5 steady state: off unless YFM_GNS5_STEADY=1
static int gns5_steady_enabled() {
  const char* e = std::getenv("YFM_GNS5_STEADY");
  return (e && e[0] == '1') ? 1 : 0;
}

// diagnostic: YFM_FZ_SPLIT_FORM=1 selects the two-function update form (FixedZFilter SPLIT_FORM)
static int split_form_enabled() {
  const char* e = std::getenv("YFM_FZ_SPLIT_FORM");
  return (e && e[0] == '1') ? 1 : 0;
}

// GNS5 initial state: two lanes per candidate (fixedz_init_coop_kernel); YFM_GNS5_INIT_LANES=1 runs the per-lane
// kernel it is bitwise equal to (tests/test_gpu_gns5_init.py).  Four lanes per candidate, at two waves per SIMD,
// measured slower (0.83 vs 0.74 ms at config 5; per-lane 1.05 ms): the replicated decode and pivot search cost more
// than the second wave hides (profiles/r6/gns5_init/).
static int gns5_init_lanes() {
  const char* e = std::getenv("YFM_GNS5_INIT_LANES");
  return (e && e[0] == '1' && e[1] == 0) ? 1 : 2;
}

template <int NP, int M, int LEAD>
static hipError_t launch_fixedz_np(const LaunchArgs& a) {
  const int grid = (a.B + kBlock - 1) / kBlock;
  if constexpr (M == 5) {
    if (!a.scratch) return hipErrorInvalidValue;
    const int ir = gns5_init_lanes();
    if (ir == 1) {
      hipLaunchKernelGGL((fixedz_init_kernel<M, LEAD>), dim3(grid), dim3(kBlock), 0, a.stream, a.theta, a.P, a.B,
                         a.space, a.scratch, a.flags_next);
    } else {
      const int gi = (int)(((size_t)a.B * 2 + kBlock - 1) / kBlock);
      hipLaunchKernelGGL((fixedz_init_coop_kernel<M, LEAD, 2>), dim3(gi), dim3(kBlock), 0, a.stream, a.theta, a.P, a.B,
                         a.space, a.scratch, a.flags_next);
    }
  }
  if (a.rec_beta) {
    hipLaunchKernelGGL((fixedz_loglik_kernel<NP, M, LEAD, true>), dim3(grid), dim3(kBlock), 0, a.stream, a.theta, a.P,
                       a.B, a.space, a.panel, a.T, a.N, a.mats, a.T_use, a.out, a.flags, a.rec_beta, a.rec_P,
                       a.horizon, a.rec_len, a.defer_list, a.defer_count, a.scratch, M == 5 ? nullptr : a.flags_next, 0);
  } else {
    constexpr bool kSteady = (M == 3 || M == 5) && (NP <= 32);  // the MFMA instantiations
    // short panels: the first (full) block and the freeze tests cost more than the steady steps save
    // (T = 34: 0.054 vs 0.045 ms; equal at T = 66; profiles/r3/probes/dns_tsweep/)
    constexpr int kSteadyMinT = 80;
    // GNS5: opt-in (YFM_GNS5_STEADY=1) — the freeze rule's contraction bound is loose for its slower closed
    // loop (spectral radius ≈ 0.74 at θ₀): almost no config-5 wave freezes, and the steady instantiation's
    // freeze tests and bound then cost 19.7 → 26.6 ms (profiles/r4/)
    const bool on = steady_enabled() && a.T >= kSteadyMinT && (M != 5 || gns5_steady_enabled());
    auto* k = (kSteady && on) ? &fixedz_loglik_kernel<NP, M, LEAD, false, kSteady>
                              : &fixedz_loglik_kernel<NP, M, LEAD, false, false>;
    // diagnostic: the two-function form of the update (commit 7a42719's regression test), GNS5 full recursion
    constexpr bool kSplitForm = (M == 5) && (NP == 30 || NP == 48);
    if constexpr (kSplitForm) {
      if (split_form_enabled()) k = &fixedz_loglik_kernel<NP, M, LEAD, false, false, true>;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, a.stream, a.theta, a.P, a.B, a.space, a.panel, a.T, a.N,
                       a.mats, a.T_use, a.out, a.flags, nullptr, nullptr, 0, 0, a.defer_list, a.defer_count,
                       a.scratch, M == 5 ? nullptr : a.flags_next, 1);
  }
  return hipGetLastError();
}

size_t fixedz_scratch_bytes(int kind, int B) {
  return kind == 2 ? sizeof(double) * (size_t)fz_rec_len<5>() * (size_t)(B > 0 ? B : 1) : 0;
}

int fixedz_np_for(int N) {
  if (N <= 8) return 8;
  if (N <= 16) return 16;
  if (N <= 24) return 24;
  if (N <= 30) return 30;
  if (N <= 32) return 32;
  if (N <= 48) return 48;
  if (N <= 64) return 64;
  return -1;
}

hipError_t launch_fixedz(int kind, const LaunchArgs& a) {
  if (kind == 0 && dns_split_supported(a.np)) {
    // the two-wave kernel (yfm_split.hip) is measured slower on MI355X: opt-in only
    const char* e = std::getenv("YFM_DNS_SPLIT");
    if (e && e[0] == '1') return launch_dns_split(a);
  }
  if (kind == 0) {
    switch (a.np) {
      case 8: return launch_fixedz_np<8, 3, 1>(a);
      case 16: return launch_fixedz_np<16, 3, 1>(a);
      case 24: return launch_fixedz_np<24, 3, 1>(a);
      case 30: return launch_fixedz_np<30, 3, 1>(a);
      case 32: return launch_fixedz_np<32, 3, 1>(a);
      case 48: return launch_fixedz_np<48, 3, 1>(a);
      case 64: return launch_fixedz_np<64, 3, 1>(a);
    }
  } else if (kind == 2) {
    switch (a.np) {
      case 8: return launch_fixedz_np<8, 5, 2>(a);
      case 16: return launch_fixedz_np<16, 5, 2>(a);
      case 24: return launch_fixedz_np<24, 5, 2>(a);
      case 30: return launch_fixedz_np<30, 5, 2>(a);
      case 32: return launch_fixedz_np<32, 5, 2>(a);
      case 48: return launch_fixedz_np<48, 5, 2>(a);
      case 64: return launch_fixedz_np<64, 5, 2>(a);
    }
  }
  return hipErrorInvalidValue;
}

hipError_t launch_prep_panel(const double* Y, int N, int T, int np, int ldp, double* out, hipStream_t s) {
  hipLaunchKernelGGL(prep_panel_kernel, dim3((T + 63) / 64), dim3(64), 0, s, Y, N, T, np, ldp, out);
  return hipGetLastError();
}

}  // namespace yfm

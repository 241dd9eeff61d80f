// yfm_tvl.hip — batched extended-Kalman-filter log-likelihood of the time-varying-λ
// DNS model (TVλDNSModel) for gfx950.
//
// Restates, per candidate θ_b:
//   get_loss                 src/models/kalman/filter.jl:182-209
//   filter! (TVλ EKF)        src/models/kalman/filter.jl:12-80
//   update_factor_loadings!  src/models/kalman/tvλdns.jl:53-64
//   initialize_filter        src/models/kalman/filter.jl:1-10
// with the reference's Jacobian column reproduced as written (filter.jl:43:
// dZ1 = z/λ − z/(λ²m), not the true derivative).
//
// Mapping: ONE FILTER PER GROUP OF L LANES.  The state is
// 4-dimensional but the loadings change every step (λ_t = 0.01 + exp(β₄)), so the
// per-step work is O(N) in the maturities: lane j of a group owns maturities
// i ≡ j (mod L), computes its share of the loadings Z (N×4), the innovation v and
// the 14 sufficient statistics of the capacitance form —
//     G = Z'Z (9 non-trivial entries; G₁₁ = N),  u = Z'v (4),  v'v (1)
// — and the group reduces them with DPP / permlane butterflies (no LDS).  Every lane
// of the group then runs the same 4×4 capacitance update redundantly, so the state
// stays replicated in VGPRs and no broadcast is needed.  L is chosen per launch so
// that B·L lanes fill the chip at two waves per SIMD (B = 16,384 → L = 8; B = 1,024 → L = 64).
//
// Capacitance form (nothing N×N is formed): B̃ = σ²I + P G, W = B̃⁻¹P,
//   K v = W u,  P_{t|t} = σ² W,  v'F⁻¹v = (v'v − u'Wu)/σ²,
//   log det F = (N−4) log σ² + log |det B̃|,  sign det F = sign det B̃.
//
// Panel: the caller's raw N×T column-major matrix (columns staged into LDS TC at a
// time, prefetched into registers one chunk ahead) plus the per-column NaN flags of
// the prepared panel (yfm_kernels.hip: prep_panel_kernel, offset np+2, stride ldp).
#include "yfm_device.hpp"
#include "yfm_internal.hpp"

namespace yfm {

namespace {

constexpr int kTvlBlock = 256;
constexpr int kTvlPre = 8;  // panel doubles prefetched per thread per chunk (≤ 2 waves/SIMD of VGPRs)

}  // namespace

// Sufficient statistics of one EKF step, indices into the accumulator array.
// Σ Z_c (c = 2..4), the Gram entries, u = Z'v and v'v, with the innovation
// v = y − Z[:,1:3]β[1:3] formed per maturity as the reference does (filter.jl:33-34): the
// uncentered reconstruction v'v = y'y − 2β'Z'y + β'Gβ loses ‖Z‖‖β‖/‖v‖ digits when the
// loadings are nearly collinear (measured: 1.8e-8 on a random N = 33, T = 3 case).
enum : int { S2 = 0, S3, S4, G22, G23, G24, G33, G34, G44, U1, U2, U3, U4, VV, NSTAT };

// Per-candidate record written by tvl_init_kernel (layout kRec* in yfm_internal.hpp): the
// decoded parameters and the initial state, so the filter kernel never holds the 10×10
// Lyapunov system in VGPRs.

// decode θ_b (transform_params + set_params!) and run initialize_filter (filter.jl:1-10)
__global__ __launch_bounds__(256) void tvl_init_kernel(const double* __restrict__ theta, int P, int B, int space,
                                                       double* __restrict__ rec, unsigned int* __restrict__ flags_next) {
  if (flags_next && blockIdx.x == 0 && threadIdx.x < kFlagsPerBank) flags_next[threadIdx.x] = 0u;  // the next launch's counters
  constexpr int M = 4;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  Params<M, 0> p;
  decode_params<M, 0>(theta + (size_t)b * P, space, p);
  double beta[M], Pm[M][M];
  const bool ok = init_state<M, 0>(p, beta, Pm);
  double* r = rec + (size_t)b * kRecLen;
  r[kRecSigma] = p.sigma2;
  int q = 0;
#pragma unroll
  for (int i = 0; i < M; ++i) {
    r[kRecDelta + i] = p.delta[i];
    r[kRecBeta + i] = beta[i];
#pragma unroll
    for (int k = 0; k < M; ++k) r[kRecPhi + i * M + k] = p.Phi[i][k];
#pragma unroll
    for (int k = i; k < M; ++k, ++q) {
      r[kRecQ + q] = p.Q[i][k];
      r[kRecP + q] = Pm[i][k];
    }
  }
  r[kRecOk] = ok ? 1.0 : 0.0;
  r[46] = 0.0;
  r[47] = 0.0;
}

// x of lane `src` of this wave (ds_bpermute: the LDS crossbar, no LDS memory and no wave barrier)
__device__ __forceinline__ double lane_read_f64(int src, double x) {
  const int lo = __builtin_amdgcn_ds_bpermute(src << 2, __double2loint(x));
  const int hi = __builtin_amdgcn_ds_bpermute(src << 2, __double2hiint(x));
  return __hiloint2double(hi, lo);
}

// Lane-distributed 4×4 update (L ≥ 4): the four roles qr = lane & 3 of each quad hold column qr of P,
// row qr of Φ, column qr of Q and δ_qr; the group's other quads repeat the same work.  Every
// quantity is formed with the replicated kernel's operation order, so the results are bitwise
// those of the one-lane-does-everything form (a role forms the upper entries (i ≤ qr) of its
// column; entries below the diagonal come from the role that owns them as upper entries, through
// the group's LDS exchange block).
struct TvlQuad {
  int qr;
  int qg;              // L ≥ 16: this quad's index in its 16-lane row
  double phq[4], qcq;  // L ≥ 16: row qg of Φ, Q[qg][qr]
  double phr[4], qc[4], dq;
  double phi[4][4];  // Φ (every row: column qr of Φ Pf)
  double* xch;  // this group's 4×4 exchange block (LDS)

  // column qr of the symmetric matrix whose upper entries are `v[i]` for i ≤ qr (this role) and
  // role k's v[qr] for k > qr; DPP: through quad exchanges instead of the LDS block (no wave barriers: the
  // latency-bound launches, L ≥ 16, take it; the throughput ones keep the fewer instructions of the LDS form)
  template <bool DPP>
  __device__ __forceinline__ void mirror(const double (&v)[4], double (&col)[4]) const {
    if constexpr (DPP) {
      quad_mirror_f64(qr, v, col);
      return;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) xch[qr * 4 + k] = v[k];
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double o = xch[k * 4 + qr];
      col[k] = k <= qr ? v[k] : o;
    }
    wave_lds_sync();  // the block is rewritten by the next exchange
  }
  // β ← δ + Φ bf;  P ← Φ Pf Φ' + Q  (propagate_state, filter.jl:162-176), from pf = column qr of the symmetric Pf:
  // role qr forms column qr of A = Φ Pf (the entry role i of the row form would form, in the same operation order),
  // one gather hands every lane A, and role qr forms column qr of A Φ' + Q
  template <bool DPP>
  __device__ __forceinline__ void propagate(const double (&bf)[4], const double (&pf)[4], double (&beta)[4],
                                            double (&Pc)[4]) const {
    double bq = dq;
#pragma unroll
    for (int j = 0; j < 4; ++j) bq = fma(phr[j], bf[j], bq);
    beta[0] = quad_bcast_f64<0>(bq);
    beta[1] = quad_bcast_f64<1>(bq);
    beta[2] = quad_bcast_f64<2>(bq);
    beta[3] = quad_bcast_f64<3>(bq);
    if constexpr (DPP) {
      // L ≥ 16: lane (qr, qg) forms entry qg of column qr of A and of the new P (role qr's ac[qg] and pc[qg], the
      // same operations); row qg of A comes from its own quad, and column qr of the new P from the lanes that formed
      // it (ds_bpermute) — a quarter of the products, four broadcasts instead of the sixteen of the 4×4 gather
      double a = 0.0;
#pragma unroll
      for (int l = 0; l < 4; ++l) a = fma(phq[l], pf[l], a);
      const double ar[4] = {quad_bcast_f64<0>(a), quad_bcast_f64<1>(a), quad_bcast_f64<2>(a), quad_bcast_f64<3>(a)};
      double t = qcq;
#pragma unroll
      for (int l = 0; l < 4; ++l) t = fma(ar[l], phr[l], t);
      const int base = (int)(threadIdx.x & 63) & ~15;
#pragma unroll
      for (int k = 0; k < 4; ++k) Pc[k] = lane_read_f64(base + (k <= qr ? 4 * k + qr : 4 * qr + k), t);
      return;
    }
    double ac[4], At[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      double a = 0.0;
#pragma unroll
      for (int l = 0; l < 4; ++l) a = fma(phi[i][l], pf[l], a);
      ac[i] = a;
    }
    quad_gather_rows<4>(ac, At);  // At[l][i] = A[i][l]
    double pc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      double t = qc[i];
#pragma unroll
      for (int l = 0; l < 4; ++l) t = fma(At[l][i], phr[l], t);
      pc[i] = t;
    }
    mirror<DPP>(pc, Pc);
  }
};

template <int L, bool RECORD>
__global__ __launch_bounds__(kTvlBlock, 2) void tvl_loglik_kernel(
    const double* __restrict__ rec, int B, const double* __restrict__ Y,
    const double* __restrict__ prep, int ldp, int np, int T, int N, int TC, const double* __restrict__ mats,
    int K, const double* __restrict__ gap_d, const int* __restrict__ gap_idx,
    const int* __restrict__ T_use, double* __restrict__ out, unsigned int* __restrict__ flags,
    double* __restrict__ rec_beta, double* __restrict__ rec_P, int horizon, int rec_len) {
  constexpr int M = 4;
  constexpr int GPB = kTvlBlock / L;  // filters per block
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double2* s_mr = reinterpret_cast<double2*>(smem);  // (m_i, 1/m_i)
  double* s_nan = smem + 2 * N;                       // TC NaN flags of the staged chunk
  double* s_y = s_nan + TC;                           // TC columns of N yields (column-major, stride N)
  double* s_w = s_y + TC * N;                         // per group: e^{-λ d_k}, k < K (≤ kTvlGaps)
  double* s_xch = s_w + GPB * kTvlGaps;               // per group: 4×4 exchange block (L ≥ 4)
  int* s_gi = reinterpret_cast<int*>(s_xch + (L >= 4 ? GPB * 16 : 0));  // gap index of the jump i → i + L
  __shared__ double s_gd[kTvlGaps];
  __shared__ int s_nobs_max;

  const int tid = threadIdx.x;
  const int j = tid % L;
  const int grp = tid / L;
  const int b = blockIdx.x * GPB + grp;
  const bool live = b < B;
  const int bb = live ? b : (B - 1);
  const int nobs = T_use ? T_use[bb] : T;

  if (tid == 0) s_nobs_max = 0;
  for (int i = tid; i < N; i += kTvlBlock) {
    const double m = mats[i];
    s_mr[i] = make_double2(m, 1.0 / m);
    if (K > 0) s_gi[i] = gap_idx[i];
  }
  if (tid < K) s_gd[tid] = gap_d[tid];
  __syncthreads();
  // loglik mode (horizon = 0) or trajectory mode (horizon ≥ 1: columns 0 .. nobs−1, then
  // horizon NaN steps — predict, filter.jl:250-282, on forecasting.jl:141's NaN padding)
  const int my_steps = horizon > 0 ? nobs + horizon : nobs - 1;
  const int my_data = horizon > 0 ? nobs : nobs - 1;
  atomicMax(&s_nobs_max, live ? my_steps : 0);

  constexpr bool DIST = L >= 4;  // distributed 4×4 update (TvlQuad)
  constexpr bool XDPP = L >= 16;  // quad transposes by DPP (TvlQuad::mirror)
  Params<M, 0> p;
  double beta[M], Pm[M][M];
  TvlQuad qd;
  double Pc[M];  // DIST: column qr of P
  bool init_ok;
  if constexpr (DIST) {
    const double* r = rec + (size_t)bb * kRecLen;
    qd.qr = tid & 3;
    qd.qg = (tid >> 2) & 3;
    qd.xch = s_xch + grp * 16;
    qd.dq = r[kRecDelta + qd.qr];
    p.sigma2 = r[kRecSigma];
#pragma unroll
    for (int i = 0; i < M; ++i) {
      beta[i] = r[kRecBeta + i];
      qd.phr[i] = r[kRecPhi + qd.qr * M + i];
#pragma unroll
      for (int k = 0; k < M; ++k) qd.phi[i][k] = r[kRecPhi + i * M + k];
      const int lo = i < qd.qr ? i : qd.qr, hi = i < qd.qr ? qd.qr : i;
      const int q = lo * M - lo * (lo - 1) / 2 + (hi - lo);  // upper-triangle record index
      qd.qc[i] = r[kRecQ + q];
      Pc[i] = r[kRecP + q];
    }
#pragma unroll
    for (int l = 0; l < M; ++l) qd.phq[l] = r[kRecPhi + qd.qg * M + l];
    {
      const int lo = qd.qg < qd.qr ? qd.qg : qd.qr, hi = qd.qg < qd.qr ? qd.qr : qd.qg;
      qd.qcq = r[kRecQ + lo * M - lo * (lo - 1) / 2 + (hi - lo)];
    }
    init_ok = r[kRecOk] != 0.0;
  } else {
    const double* r = rec + (size_t)bb * kRecLen;
    p.sigma2 = r[kRecSigma];
    int q = 0;
#pragma unroll
    for (int i = 0; i < M; ++i) {
      p.delta[i] = r[kRecDelta + i];
      beta[i] = r[kRecBeta + i];
#pragma unroll
      for (int k = 0; k < M; ++k) p.Phi[i][k] = r[kRecPhi + i * M + k];
#pragma unroll
      for (int k = i; k < M; ++k, ++q) {
        p.Q[i][k] = p.Q[k][i] = r[kRecQ + q];
        Pm[i][k] = Pm[k][i] = r[kRecP + q];
      }
    }
    init_ok = r[kRecOk] != 0.0;
  }
  (void)Pc;
  double l_minm = __builtin_inf();  // this lane's smallest maturity (the λ-overflow test below)
  for (int i = j; i < N; i += L) l_minm = fmin(l_minm, s_mr[i].x);
  const double sigma2 = p.sigma2;
  const double rsig2 = 1.0 / sigma2;

  LogDetAcc ld;
  double sumq = 0.0;
  bool neg = false;
  double last_det = 0.0, last_q = 0.0;  // fresh model: F = 0, F⁻¹ = 0, v = 0 (kalmanbasemodel.jl:65-67)

  __syncthreads();
  const int nsteps = max(s_nobs_max, 0);
  const int CHY = TC * N;  // yields per chunk

  // ---- panel staging: chunk c (columns cTC .. cTC+TC-1) in LDS, chunk c+1 in registers ----
  double pre[kTvlPre];
  double pre_nan = 0.0;
  auto load_chunk = [&](int c) {
    const size_t base = (size_t)c * CHY;
    const size_t lim = (size_t)T * N;
#pragma unroll
    for (int r = 0; r < kTvlPre; ++r) {
      const int e = r * kTvlBlock + tid;
      const size_t g = base + e;
      pre[r] = (e < CHY && g < lim) ? Y[g] : 0.0;
    }
    const int tc = c * TC + tid;
    pre_nan = (tid < TC && tc < T) ? prep[(size_t)tc * ldp + np + 2] : 0.0;
  };
  auto store_chunk = [&]() {
#pragma unroll
    for (int r = 0; r < kTvlPre; ++r) {
      const int e = r * kTvlBlock + tid;
      if (e < CHY) s_y[e] = pre[r];
    }
    if (tid < TC) s_nan[tid] = pre_nan;
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
    const bool act = live && t < my_steps;  // the tail block's padding groups skip the filter (B = 1: three of four waves)
    const bool acc = t >= 1;  // Julia t > 1 (filter.jl:194)
    const bool nan_col = nan_next != 0.0 || t >= my_data;
    if (tt + 1 < TC) nan_next = s_nan[tt + 1];  // the next chunk's first flag is read after its store
    if (act && nan_col) {
      // filter.jl:13-29: prediction only; F, F⁻¹, v stale → the loglik re-adds the last term
      if constexpr (DIST) {
        double bf[M], pf[M];
#pragma unroll
        for (int i = 0; i < M; ++i) {
          bf[i] = beta[i];
          pf[i] = Pc[i];
        }
        qd.propagate<XDPP>(bf, pf, beta, Pc);
      } else {
        double bf[M], Pf[M][M];
#pragma unroll
        for (int i = 0; i < M; ++i) {
          bf[i] = beta[i];
#pragma unroll
          for (int k = i; k < M; ++k) Pf[i][k] = Pm[i][k];
        }
        propagate_state<M, 0>(p, bf, Pf, beta, Pm);
      }
      if (acc) {
        ld.mul(last_det);
        sumq += last_q;
        neg = neg || (last_det < 0.0);
      }
    } else if (act) {
      // ---- loadings and sufficient statistics over this lane's maturities ----
      const double lam = 1e-2 + exp(beta[3]);  // tvλdns.jl:56
      const double rl = 1.0 / lam;
      const double dl = lam - 1e-2;            // filter.jl:38
      // λ near the FP64 range: every z = e^{−λm} of this lane underflows to 0 (λ·m_min > 746, or c1 or c2
      // overflows) and the reference's Jacobian column is ((β2+β3)·0 + β3·0)·dλ = 0·dλ (0, or NaN for
      // dλ = Inf), so the factored form's constants become 0·dλ instead of multiplying z = 0 by an Inf
      // (c2·m can overflow with c2 itself finite: randomized sweep case 4985, λ = 3.6e304)
      const double c1r = (beta[1] + beta[2]) * dl, c2r = beta[2] * dl;
      const bool big = !(lam * l_minm <= 746.0) || !(fabs(c1r) <= __DBL_MAX__) || !(fabs(c2r) <= __DBL_MAX__);
      const double c1 = big ? 0.0 * dl : c1r;
      const double c2 = big ? 0.0 * dl : c2r;
      const double k1 = c1 * rl;
      const double* col = s_y + tt * N;
      double s[NSTAT];
#pragma unroll
      for (int k = 0; k < NSTAT; ++k) s[k] = 0.0;
      // one maturity: z = e^{-λm}, loadings, Jacobian column, statistics
      auto accum = [&](double2 mr, double z, double y) {
        const double m = mr.x;
        const double it = rl * mr.y;             // 1/τ
        const double z2 = (1.0 - z) * it;        // (1 − z)/τ
        const double z3 = z2 - z;
        // Jacobian column as written (filter.jl:43-46): ((β2+β3)(z/λ − z/(λ²m)) + β3·m·z)·(λ − 0.01)
        //   = z·(k1 − k1/(λm) + c2·m),  k1 = c1/λ
        const double z4 = z * fma(c2, m, fma(-k1, it, k1));
        s[S2] += z2;
        s[S3] += z3;
        s[S4] += z4;
        s[G22] = fma(z2, z2, s[G22]);
        s[G23] = fma(z2, z3, s[G23]);
        s[G24] = fma(z2, z4, s[G24]);
        s[G33] = fma(z3, z3, s[G33]);
        s[G34] = fma(z3, z4, s[G34]);
        s[G44] = fma(z4, z4, s[G44]);
        const double v = y - fma(beta[2], z3, fma(beta[1], z2, beta[0]));  // y − Z[:,1:3]β[1:3]
        s[U1] += v;
        s[U2] = fma(z2, v, s[U2]);
        s[U3] = fma(z3, v, s[U3]);
        s[U4] = fma(z4, v, s[U4]);
        s[VV] = fma(v, v, s[VV]);
      };
      if (K > 0) {
        // few distinct jumps d_k = m_{i+L} − m_i: z_{i+L} = z_i · e^{-λ d_k}, one exp per lane
        // plus K per group instead of one per maturity (relative drift ≤ (N/L) ulp)
        double z = (j < N) ? exp(-(lam * s_mr[j].x)) : 0.0;
        if (K == 1) {
          // one jump (uniform grids): every lane forms the factor itself — the same exp of the same argument,
          // with no LDS round trip and wave barrier on the step's serial path
          const double wn = exp(-(lam * s_gd[0]));
#pragma unroll 2
          for (int i = j; i < N; i += L) {
            accum(s_mr[i], z, col[i]);
            z *= wn;
          }
        } else {
          double* w = s_w + grp * kTvlGaps;
          for (int q = j; q < K; q += L) w[q] = exp(-(lam * s_gd[q]));
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 2
          for (int i = j; i < N; i += L) {
            const double2 mr = s_mr[i];
            const double wn = w[s_gi[i]];
            accum(mr, z, col[i]);
            z *= wn;
          }
        }
      } else {
#pragma unroll 2
        for (int i = j; i < N; i += L) {
          const double2 mr = s_mr[i];
          accum(mr, exp(-(lam * mr.x)), col[i]);  // z_i = e^{-τ_i}
        }
      }
#pragma unroll
      for (int k = 0; k < NSTAT; ++k) s[k] = group_sum<L>(s[k]);

      double G[M][M];
      G[0][0] = (double)N;
      G[0][1] = G[1][0] = s[S2];
      G[0][2] = G[2][0] = s[S3];
      G[0][3] = G[3][0] = s[S4];
      G[1][1] = s[G22];
      G[1][2] = G[2][1] = s[G23];
      G[1][3] = G[3][1] = s[G24];
      G[2][2] = s[G33];
      G[2][3] = G[3][2] = s[G34];
      G[3][3] = s[G44];
      const double u[M] = {s[U1], s[U2], s[U3], s[U4]};
      const double vv = s[VV];

      double det, q;
      bool upd;
      if constexpr (DIST) {
        // row qr of B̃ = σ²I + P G (P symmetric: row qr is the column this role holds), broadcast
        double Ar[M], A[M][M], x[M];
#pragma unroll
        for (int k = 0; k < M; ++k) {
          double t = (k == qd.qr) ? sigma2 : 0.0;
#pragma unroll
          for (int l = 0; l < M; ++l) t = fma(Pc[l], G[l][k], t);
          Ar[k] = t;
          x[k] = Pc[k];
        }
        quad_gather_rows<M>(Ar, A);
        // Capacitance::solve with ONE right-hand side: column qr of P
        double sgn = 1.0, prod = 1.0;
#pragma unroll
        for (int k = 0; k < M; ++k) {
          int pv = k;
          double amax = fabs(A[k][k]);
#pragma unroll
          for (int i = k + 1; i < M; ++i) {
            const double a = fabs(A[i][k]);
            const bool gt = a > amax;
            amax = gt ? a : amax;
            pv = gt ? i : pv;
          }
          sgn = (pv != k) ? -sgn : sgn;
#pragma unroll
          for (int i = k + 1; i < M; ++i) {
            const bool sw = (pv == i);
#pragma unroll
            for (int c = k; c < M; ++c) {
              const double a = A[k][c], b = A[i][c];
              A[k][c] = sw ? b : a;
              A[i][c] = sw ? a : b;
            }
            const double a = x[k], b = x[i];
            x[k] = sw ? b : a;
            x[i] = sw ? a : b;
          }
          const double piv = A[k][k];
          prod *= piv;
          const double rp = 1.0 / piv;
#pragma unroll
          for (int i = k + 1; i < M; ++i) {
            const double l = A[i][k] * rp;
#pragma unroll
            for (int c = k + 1; c < M; ++c) A[i][c] = fma(-l, A[k][c], A[i][c]);
            x[i] = fma(-l, x[k], x[i]);
          }
        }
#pragma unroll
        for (int k = M - 1; k >= 0; --k) {
          const double rp = 1.0 / A[k][k];
          double t = x[k];
#pragma unroll
          for (int j2 = k + 1; j2 < M; ++j2) t = fma(-A[k][j2], x[j2], t);
          x[k] = t * rp;
        }
        det = sgn * prod;
        // column qr of W (its upper triangle mirrored, as the replicated form uses it)
        double wc[M];
        qd.mirror<XDPP>(x, wc);
        double wq = 0.0;
#pragma unroll
        for (int k = 0; k < M; ++k) wq = fma(wc[k], u[k], wq);
        const double w[M] = {quad_bcast_f64<0>(wq), quad_bcast_f64<1>(wq), quad_bcast_f64<2>(wq), quad_bcast_f64<3>(wq)};
        double bf[M], uk = 0.0;
#pragma unroll
        for (int i = 0; i < M; ++i) {
          bf[i] = beta[i] + w[i];
          uk = fma(u[i], w[i], uk);
        }
        q = (vv - uk) * rsig2;
        upd = det != 0.0;  // inv(F) threw: return without updating (filter.jl:51-56)
        if (upd) {
          double pfc[M];
#pragma unroll
          for (int k = 0; k < M; ++k) pfc[k] = sigma2 * wc[k];
          qd.propagate<XDPP>(bf, pfc, beta, Pc);
        }
      } else {
      double W[M][M];
      Capacitance<M>::solve(Pm, G, sigma2, W, det);
#pragma unroll
      for (int i = 0; i < M; ++i)
#pragma unroll
        for (int k = 0; k < i; ++k) W[i][k] = W[k][i];
      double bf[M], Pf[M][M], uk = 0.0;
#pragma unroll
      for (int i = 0; i < M; ++i) {
        double w = 0.0;
#pragma unroll
        for (int k = 0; k < M; ++k) w = fma(W[i][k], u[k], w);
        bf[i] = beta[i] + w;
        uk = fma(u[i], w, uk);
      }
      q = (vv - uk) * rsig2;
#pragma unroll
      for (int i = 0; i < M; ++i)
#pragma unroll
        for (int k = i; k < M; ++k) Pf[i][k] = sigma2 * W[i][k];
      upd = det != 0.0;  // inv(F) threw: return without updating (filter.jl:51-56)
      if (upd) propagate_state<M, 0>(p, bf, Pf, beta, Pm);
      }
      last_det = det;
      last_q = upd ? q : __builtin_nan("");
      if (acc) {
        ld.mul(det);
        sumq += last_q;
        neg = neg || (det < 0.0);
      }
    }
    if constexpr (RECORD) {
      double Pfull[M][M];
      if constexpr (DIST) quad_gather_rows<M>(Pc, Pfull);  // every lane of the quad takes part
      const int slot = t - max(0, my_steps - rec_len);  // the last rec_len steps
      if (live && act && j == 0 && slot >= 0) {
        const size_t o = (size_t)b * (size_t)rec_len + slot;
#pragma unroll
        for (int i = 0; i < M; ++i) rec_beta[o * M + i] = beta[i];
        if (rec_P) {
#pragma unroll
          for (int k = 0; k < M; ++k)
#pragma unroll
            for (int i = 0; i < M; ++i) rec_P[o * M * M + k * M + i] = DIST ? Pfull[i][k] : Pm[i][k];
        }
      }
    }
    if (tt == TC - 1) {  // chunk done: its buffer takes the prefetched chunk, prefetch the one after
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
    ll = __builtin_nan("");  // the reference throws from initialize_filter
    atomicAdd(&flags[0], 1u);
  } else {
    const int nterms = max(nobs - 2, 0);
    if (nterms == 0) {
      ll = 0.0;
    } else {
      const double per_term = (double)(N - M) * log(sigma2) + (double)N * kLog2Pi;
      ll = -0.5 * ((double)nterms * per_term + ld.log_value() + sumq);
    }
    if (neg || !isfinite(ll)) {  // DomainError / non-finite → -Inf (filter.jl:197-204)
      ll = -__builtin_inf();
      atomicAdd(&flags[1], 1u);
    }
  }
  out[b] = ll;
}

namespace {

template <int L>
hipError_t launch_tvl_l(const LaunchArgs& a, const TvlGaps& g, int TC) {
  constexpr int GPB = kTvlBlock / L;
  const int grid = (a.B + GPB - 1) / GPB;
  const size_t shmem = sizeof(double) * (size_t)(2 * a.N + TC + TC * a.N + GPB * kTvlGaps + (L >= 4 ? GPB * 16 : 0)) +
                       sizeof(int) * a.N;
  hipLaunchKernelGGL(tvl_init_kernel, dim3((a.B + 255) / 256), dim3(256), 0, a.stream, a.theta, a.P, a.B, a.space,
                     a.scratch, a.flags_next);
  if (a.rec_beta) {
    hipLaunchKernelGGL((tvl_loglik_kernel<L, true>), dim3(grid), dim3(kTvlBlock), shmem, a.stream, a.scratch, a.B,
                       a.raw, a.panel, a.ldp, a.np, a.T, a.N, TC, a.mats, g.K, g.d, g.idx, a.T_use, a.out, a.flags, a.rec_beta,
                       a.rec_P, a.horizon, a.rec_len);
  } else {
    hipLaunchKernelGGL((tvl_loglik_kernel<L, false>), dim3(grid), dim3(kTvlBlock), shmem, a.stream, a.scratch, a.B,
                       a.raw, a.panel, a.ldp, a.np, a.T, a.N, TC, a.mats, g.K, g.d, g.idx, a.T_use, a.out, a.flags, nullptr,
                       nullptr, 0, 0);
  }
  return hipGetLastError();
}

}  // namespace

size_t tvl_scratch_bytes(int B) { return sizeof(double) * (size_t)kRecLen * (size_t)(B > 0 ? B : 1); }

int tvl_max_n() { return (kTvlPre * kTvlBlock) - 1; }

int tvl_lanes_for(int B, int N, int share) {
  // The L (a power of two ≤ 64, ≤ the maturity count rounded up) with the least modelled time.  Per filter step a
  // wave issues ≈ ⌈N/L⌉·28 instructions of maturity loop, ≈ 1,450 of 4×4 update and per-step constants (replicated
  // on every lane of a group) and ≈ 60 per butterfly level; the kernel holds two waves per SIMD (2,048 on the chip)
  // and issues at ≈ 0.7 of that rate with one (L = 4 vs 8 at B = 16,384, N = 360: 6.06 vs 5.77 ms,
  // profiles/r1/final/tvl_lanes).  `share` concurrent launches of this size divide the SIMDs.  Measured choices it
  // keeps at N = 360: B = 16,384 → 8, B = 65,536 → 2, B ≤ 1,024 → 64.  At N = 30 the update dominates: the
  // estimator's 7,680-point rounds take L = 4 (the round-4 rule, "fill two waves per SIMD", gave 32).
  int capN = 1;
  while (capN < N && capN < 64) capN <<= 1;
  const double waves_per_simd_unit = (double)(B > 0 ? B : 1) * (share > 0 ? share : 1) / (64.0 * 1024.0);
  int best = 1;
  double best_cost = 0.0;
  for (int L = 1, lg = 0; L <= capN; L <<= 1, ++lg) {
    const double wps = waves_per_simd_unit * L;  // waves per SIMD
    const double issue = (double)((N + L - 1) / L) * 28.0 + 1450.0 + 60.0 * lg;
    const double eff = wps >= 2.0 ? 1.0 : (wps <= 1.0 ? 0.7 : 0.7 + 0.3 * (wps - 1.0));
    const double cost = (wps > 1.0 ? wps : 1.0) * issue / eff;
    if (L == 1 || cost < best_cost) {
      best = L;
      best_cost = cost;
    }
  }
  return best;
}

hipError_t launch_tvl(const LaunchArgs& a, const TvlGaps& g, int lanes) {
  // columns per chunk: the prefetch registers hold ≤ kTvlPre·256 yields
  int TC = (kTvlPre * kTvlBlock) / a.N;
  if (TC > 32) TC = 32;
  if (TC < 1) return hipErrorInvalidValue;
  switch (lanes) {
    case 1: return launch_tvl_l<1>(a, g, TC);
    case 2: return launch_tvl_l<2>(a, g, TC);
    case 4: return launch_tvl_l<4>(a, g, TC);
    case 8: return launch_tvl_l<8>(a, g, TC);
    case 16: return launch_tvl_l<16>(a, g, TC);
    case 32: return launch_tvl_l<32>(a, g, TC);
    case 64: return launch_tvl_l<64>(a, g, TC);
  }
  return hipErrorInvalidValue;
}

}  // namespace yfm

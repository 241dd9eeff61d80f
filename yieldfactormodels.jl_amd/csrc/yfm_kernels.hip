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
// Lanes whose Z'Z is numerically singular (N < M, or λ so large that Z's columns
// collapse) take the CAPACITANCE form instead: B̃ = σ²I + PG, pivoted LU,
// W = B̃⁻¹P, v'F⁻¹v = (v'v − u'Wu)/σ², P_{t|t} = σ²W, log det F = (N−M) log σ² +
// log det B̃.
//
// Panel layout in HBM (built by prep_panel_kernel from the caller's N×T
// column-major matrix): T columns of LDP = NP + 4 doubles —
//   [ ỹ_0 … ỹ_{N-1}, 0 … 0 (to NP), ȳ, ỹ'ỹ, isnan(any y), y'y ].
#include "yfm_device.hpp"

namespace yfm {

constexpr int kBlock = 256;  // 4 waves: one per SIMD of a CU
constexpr int kTC = 32;      // panel columns per LDS chunk

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

// Fixed-loading models: DNS (M = 3, one γ, dns.jl:51-65) and the 5-factor
// generalised NS extension (M = 5, two γ; SURVEY §8 a9, not in the reference).
// Z column 0 is ones; columns 1.. come in (slope, curvature) pairs per γ:
// S = (1 − e^{−λm})/(λm), C = S − e^{−λm}.
template <int NP, int M, int LEAD, bool RECORD>
__global__ __launch_bounds__(kBlock, 1) void fixedz_loglik_kernel(
    const double* __restrict__ theta, int P, int B, int space, const double* __restrict__ panel, int T, int N,
    const double* __restrict__ mats, const int* __restrict__ T_use, double* __restrict__ out,
    unsigned int* __restrict__ flags, double* __restrict__ rec_beta, double* __restrict__ rec_P) {
  constexpr int LDP = NP + 4;
  constexpr int CH = kTC * LDP;               // doubles per chunk
  constexpr int PER = (CH + kBlock - 1) / kBlock;
  constexpr int NZ = M - 1;                   // non-constant loading columns
  static_assert(NZ == 2 * LEAD, "loading columns come in (S, C) pairs per gamma");
  __shared__ __attribute__((aligned(16))) double sh[2][CH];
  __shared__ int s_nobs_max;

  const int tid = threadIdx.x;
  const int b = blockIdx.x * kBlock + tid;
  const bool live = b < B;
  const int bb = live ? b : (B - 1);
  const int nobs = T_use ? T_use[bb] : T;

  if (tid == 0) s_nobs_max = 0;
  __syncthreads();
  atomicMax(&s_nobs_max, live ? nobs : 0);

  // ---- decode θ_b, loadings, Z'Z, initial state ----------------------------------
  Params<M, LEAD> p;
  decode_params<M, LEAD>(theta + (size_t)bb * P, space, p);

  double Zc[NZ][NP];
#pragma unroll
  for (int l = 0; l < LEAD; ++l) {
    const double lam = 1e-2 + exp(p.gam[l]);  // dns.jl:55
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      if (i < N) {
        const double tau = lam * mats[i];
        const double z = exp(-tau);
        const double s = (1.0 - z) / tau;
        Zc[2 * l][i] = s;
        Zc[2 * l + 1][i] = s - z;
      } else {
        Zc[2 * l][i] = 0.0;
        Zc[2 * l + 1][i] = 0.0;
      }
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
  const double sigma2 = p.sigma2;
  const double rsig2 = 1.0 / sigma2;

  // G⁻¹ (pivoted elimination) and log det G; decide collapsed vs capacitance per lane.
  double R[M][M];
  double logdetG = 0.0;
  bool collapsed;
  {
    double A[M][M], X[M][M];
    double hadamard = 1.0;
#pragma unroll
    for (int i = 0; i < M; ++i) {
      hadamard *= G[i][i];
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
    // Z'Z must be numerically nonsingular: det / ∏ diag (Hadamard ratio, ≤ 1).
    collapsed = ok && (N >= M) && (detG > 1e-13 * hadamard);
    logdetG = collapsed ? log(detG) : 0.0;
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
      for (int j = 0; j < M; ++j) R[i][j] = sigma2 * 0.5 * (X[i][j] + X[j][i]);
  }
  // Gi·(0, z̃) only needs the columns 1.. of G⁻¹ = R/σ²

  double beta[M], Pm[M][M];
  const bool init_ok = init_state<M, LEAD>(p, beta, Pm);

  LogDetAcc ld;
  double sumq = 0.0;
  bool neg = false;
  double last_det = 0.0, last_q = 0.0;  // fresh model: F = 0, F⁻¹ = 0, v = 0 (kalmanbasemodel.jl:65-67)

  __syncthreads();
  const int nsteps = max(s_nobs_max - 1, 0);
  const int my_steps = nobs - 1;
  const int nchunks = (nsteps + kTC - 1) / kTC;

  double pre[PER];
  auto load_chunk = [&](int c) {
    const size_t base = (size_t)c * CH;
    const size_t lim = (size_t)T * LDP;
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      const int e = r * kBlock + tid;
      const size_t g = base + e;
      pre[r] = (e < CH && g < lim) ? panel[g] : 0.0;
    }
  };
  if (nchunks > 0) load_chunk(0);

  for (int c = 0; c < nchunks; ++c) {
    double* buf = sh[c & 1];
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      const int e = r * kBlock + tid;
      if (e < CH) buf[e] = pre[r];
    }
    __syncthreads();
    if (c + 1 < nchunks) load_chunk(c + 1);

    const int tend = min(kTC, nsteps - c * kTC);
    for (int tt = 0; tt < tend; ++tt) {
      const int t = c * kTC + tt;  // 0-based step; reads column t (Julia t+1)
      const double* col = buf + tt * LDP;
      const double2 meta = *reinterpret_cast<const double2*>(col + NP + 2);  // (nanflag, y'y)
      const bool act = t < my_steps;
      if (!act) continue;
      const bool acc = t >= 1;  // Julia t > 1 (filter.jl:194)

      if (meta.x != 0.0) {
        // NaN column: prediction only (filter.jl:126-140); F, v stale → the loglik
        // re-adds the previous term (filter.jl:195 reads base.F / base.v unchanged).
        double nb[M];
#pragma unroll
        for (int i = 0; i < M; ++i) {
          double s = p.delta[i];
#pragma unroll
          for (int j = 0; j < M; ++j) s = fma(p.Phi[i][j], beta[j], s);
          nb[i] = s;
        }
        double A[M][M];
#pragma unroll
        for (int i = 0; i < M; ++i)
#pragma unroll
          for (int j = 0; j < M; ++j) {
            double s = 0.0;
#pragma unroll
            for (int l = 0; l < M; ++l) s = fma(p.Phi[i][l], Pm[l][j], s);
            A[i][j] = s;
          }
#pragma unroll
        for (int i = 0; i < M; ++i) {
          beta[i] = nb[i];
#pragma unroll
          for (int j = i; j < M; ++j) {
            double s = p.Q[i][j];
#pragma unroll
            for (int l = 0; l < M; ++l) s = fma(A[i][l], p.Phi[j][l], s);
            Pm[i][j] = s;
            Pm[j][i] = s;
          }
        }
        if (acc) {
          ld.mul(last_det);
          sumq += last_q;
          neg = neg || (last_det < 0.0);
        }
      } else {
        // ---- z̃ = Z'ỹ_t for the non-constant columns (Σỹ = 0) ----
        const double2 yb = *reinterpret_cast<const double2*>(col + NP);  // (ȳ, ỹ'ỹ)
        double zt[NZ];
        {
          double a[NZ][2];
#pragma unroll
          for (int cz = 0; cz < NZ; ++cz) { a[cz][0] = 0.0; a[cz][1] = 0.0; }
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
        double det, q;
        double bf[M];   // β_{t|t}
        double Pf[M][M];  // P_{t|t}
        if (collapsed) {
          // ĉ = G⁻¹ (0, z̃) + ȳ e₀ ;  r'r = ỹ'ỹ − z̃'ĉ[1:]
          double ch[M];
#pragma unroll
          for (int i = 0; i < M; ++i) {
            double s = 0.0;
#pragma unroll
            for (int j = 1; j < M; ++j) s = fma(R[i][j], zt[j - 1], s);
            ch[i] = s * rsig2;
          }
          double rr = yb.y;
#pragma unroll
          for (int j = 1; j < M; ++j) rr = fma(-zt[j - 1], ch[j], rr);
          ch[0] += yb.x;
          double S[M][M];
          double X[M][M + 1];  // [c | R] → [S⁻¹c | S⁻¹R]
#pragma unroll
          for (int i = 0; i < M; ++i) {
#pragma unroll
            for (int j = 0; j < M; ++j) {
              S[i][j] = Pm[i][j] + R[i][j];
              X[i][j + 1] = R[i][j];
            }
            X[i][0] = ch[i] - beta[i];
          }
          det = ldlt_solve<M, M + 1>(S, X);
          double cx = 0.0;
#pragma unroll
          for (int i = 0; i < M; ++i) cx = fma(ch[i] - beta[i], X[i][0], cx);
          q = fma(rr, rsig2, cx);
#pragma unroll
          for (int i = 0; i < M; ++i) {
            double s = beta[i];
#pragma unroll
            for (int k = 0; k < M; ++k) s = fma(Pm[i][k], X[k][0], s);
            bf[i] = s;
          }
#pragma unroll
          for (int i = 0; i < M; ++i)
#pragma unroll
            for (int j = i; j < M; ++j) {
              double s = 0.0;
#pragma unroll
              for (int k = 0; k < M; ++k) s = fma(Pm[i][k], X[k][j + 1], s);
              Pf[i][j] = s;
              Pf[j][i] = s;
            }
        } else {
          // capacitance form on uncentered sums: Z'y = (Nȳ, z̃ + ȳ G[1:,0]), y'y
          double zy[M];
          zy[0] = (double)N * yb.x;
#pragma unroll
          for (int j = 1; j < M; ++j) zy[j] = fma(yb.x, G[j][0], zt[j - 1]);
          double u[M];
          double bgb = 0.0, bzy = 0.0;
#pragma unroll
          for (int i = 0; i < M; ++i) {
            double g = 0.0;
#pragma unroll
            for (int j = 0; j < M; ++j) g = fma(G[i][j], beta[j], g);
            u[i] = zy[i] - g;
            bgb = fma(beta[i], g, bgb);
            bzy = fma(beta[i], zy[i], bzy);
          }
          const double vv = fma(-2.0, bzy, meta.y) + bgb;
          double W[M][M];
          Capacitance<M>::solve(Pm, G, sigma2, W, det);
#pragma unroll
          for (int i = 0; i < M; ++i)
#pragma unroll
            for (int j = 0; j < i; ++j) W[i][j] = W[j][i];
          double uk = 0.0;
#pragma unroll
          for (int i = 0; i < M; ++i) {
            double s = 0.0;
#pragma unroll
            for (int j = 0; j < M; ++j) s = fma(W[i][j], u[j], s);
            bf[i] = beta[i] + s;
            uk = fma(u[i], s, uk);
          }
          q = (vv - uk) * rsig2;
#pragma unroll
          for (int i = 0; i < M; ++i)
#pragma unroll
            for (int j = 0; j < M; ++j) Pf[i][j] = sigma2 * W[i][j];
        }

        const bool upd = !(t == 0 && det == 0.0);  // inv(F) threw at t=1: skip update (filter.jl:151-154)
        if (upd) {
#pragma unroll
          for (int i = 0; i < M; ++i) {  // β ← δ + Φ β_{t|t}   (filter.jl:162-165)
            double s = p.delta[i];
#pragma unroll
            for (int j = 0; j < M; ++j) s = fma(p.Phi[i][j], bf[j], s);
            beta[i] = s;
          }
          // P ← Φ P_{t|t} Φ' + Q   (≡ Φ(I − KZ)PΦ' + Q, filter.jl:168-176)
          double A[M][M];
#pragma unroll
          for (int i = 0; i < M; ++i)
#pragma unroll
            for (int j = 0; j < M; ++j) {
              double s = 0.0;
#pragma unroll
              for (int l = 0; l < M; ++l) s = fma(p.Phi[i][l], Pf[l][j], s);
              A[i][j] = s;
            }
#pragma unroll
          for (int i = 0; i < M; ++i)
#pragma unroll
            for (int j = i; j < M; ++j) {
              double s = p.Q[i][j];
#pragma unroll
              for (int l = 0; l < M; ++l) s = fma(A[i][l], p.Phi[j][l], s);
              Pm[i][j] = s;
              Pm[j][i] = s;
            }
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
        if (live) {
          const size_t o = (size_t)b * (size_t)(T - 1) + t;
#pragma unroll
          for (int i = 0; i < M; ++i) rec_beta[o * M + i] = beta[i];
#pragma unroll
          for (int j = 0; j < M; ++j)
#pragma unroll
            for (int i = 0; i < M; ++i) rec_P[o * M * M + j * M + i] = Pm[i][j];
        }
      }
    }
  }

  if (!live) return;
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
      ll = -0.5 * ((double)nterms * per_term + ld.log_value() + sumq);
    }
    if (neg || !isfinite(ll)) {  // DomainError / non-finite → -Inf (filter.jl:197-204)
      ll = -__builtin_inf();
      atomicAdd(&flags[1], 1u);
    }
  }
  out[b] = ll;
}

}  // namespace yfm

// ------------------------------------------------------------------------------------
// host-side dispatch (declared in yfm_internal.hpp)
// ------------------------------------------------------------------------------------
#include "yfm_internal.hpp"

namespace yfm {

template <int NP, int M, int LEAD>
static hipError_t launch_fixedz_np(const LaunchArgs& a) {
  const int grid = (a.B + kBlock - 1) / kBlock;
  if (a.rec_beta) {
    hipLaunchKernelGGL((fixedz_loglik_kernel<NP, M, LEAD, true>), dim3(grid), dim3(kBlock), 0, a.stream, a.theta, a.P,
                       a.B, a.space, a.panel, a.T, a.N, a.mats, a.T_use, a.out, a.flags, a.rec_beta, a.rec_P);
  } else {
    hipLaunchKernelGGL((fixedz_loglik_kernel<NP, M, LEAD, false>), dim3(grid), dim3(kBlock), 0, a.stream, a.theta,
                       a.P, a.B, a.space, a.panel, a.T, a.N, a.mats, a.T_use, a.out, a.flags, nullptr, nullptr);
  }
  return hipGetLastError();
}

int fixedz_np_for(int N) {
  if (N <= 8) return 8;
  if (N <= 16) return 16;
  if (N <= 24) return 24;
  if (N <= 32) return 32;
  if (N <= 48) return 48;
  if (N <= 64) return 64;
  return -1;
}

hipError_t launch_fixedz(int kind, const LaunchArgs& a) {
  if (kind == 0) {
    switch (a.np) {
      case 8: return launch_fixedz_np<8, 3, 1>(a);
      case 16: return launch_fixedz_np<16, 3, 1>(a);
      case 24: return launch_fixedz_np<24, 3, 1>(a);
      case 32: return launch_fixedz_np<32, 3, 1>(a);
      case 48: return launch_fixedz_np<48, 3, 1>(a);
      case 64: return launch_fixedz_np<64, 3, 1>(a);
    }
  } else if (kind == 2) {
    switch (a.np) {
      case 8: return launch_fixedz_np<8, 5, 2>(a);
      case 16: return launch_fixedz_np<16, 5, 2>(a);
      case 24: return launch_fixedz_np<24, 5, 2>(a);
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

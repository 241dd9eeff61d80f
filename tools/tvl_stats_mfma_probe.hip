// tvl_stats_mfma_probe.hip — the per-step statistics phase of the TVλ EKF (config 3: N = 360
// maturities, T = 600 steps, B = 16,384 filters) in two formulations, to decide whether the
// Gram / innovation contraction belongs on the matrix cores:
//
//   VALU  (what csrc/yfm_tvl.hip runs): one filter per group of L = 8 lanes, lane j owns the
//         maturities i ≡ j (mod 8); per maturity it forms z, the loadings (z2, z3, z4), the
//         innovation v and FMA-accumulates the 14 statistics (Σz_c, Z'Z, Z'v, v'v); the group
//         reduces them with DPP butterflies.
//   MFMA  v_mfma_f64_4x4x4_4b_f64: four filters per wave, one per block of 16 lanes; lane
//         (k, blk, x) supplies column x of maturity 4c + k of its filter (A = [1 z2 z3 z4],
//         B = [v z2 z3 z4]), so one instruction accumulates D = AᵀB (Z'Z, Z'v) over four
//         maturities of four filters; v'v is a VALU FMA on the x = 0 lanes.  Each column value
//         is formed in the cheapest uniform way, z·(a + b/m + c·m) + d/m + e + f·y with per-lane
//         coefficients, so no lane selects between formulas.
//
// The loadings must be formed per maturity and step either way (λ_t follows the filtered state);
// the MFMA layout makes four lanes form four columns of one maturity where the VALU form lets one
// lane form all of them, so the question is whether the matrix cores' 14 saved FMAs per maturity
// outweigh that.  Both kernels stage panel columns in LDS identically and write per-filter
// checksums of every statistic (compared to ~1e-12).
// Build: hipcc --offload-arch=gfx950 -O3 tvl_stats_mfma_probe.hip -o tvl_stats_mfma_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

constexpr int N = 360, T = 600, B = 16384, TC = 16, BLK = 256;
constexpr int NSTAT = 15;  // S1(=N) S2 S3 S4 G22 G23 G24 G33 G34 G44 U1 U2 U3 U4 VV (S1 kept for layout)

__device__ __forceinline__ void filter_consts(int b, int t, double (&beta)[4]) {
  const double ph = 0.1 * t + 0.37 * b;
  beta[0] = 5.0 + 0.1 * sin(ph);
  beta[1] = -1.5 + 0.1 * cos(ph);
  beta[2] = 0.5 + 0.05 * sin(1.3 * ph);
  beta[3] = log(0.0509) + 0.05 * cos(0.7 * ph);
}

template <int LVL>
__device__ __forceinline__ double lvl_sum(double x) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  constexpr int ctrl = LVL == 0 ? 0xB1 : LVL == 1 ? 0x4E : 0x141;
  const int plo = __builtin_amdgcn_update_dpp(0, lo, ctrl, 0xf, 0xf, false);
  const int phi = __builtin_amdgcn_update_dpp(0, hi, ctrl, 0xf, 0xf, false);
  return x + __hiloint2double(phi, plo);
}

__device__ __forceinline__ void stage(const double* __restrict__ Y, double* s_y, int t0) {
  __syncthreads();
  for (int e = threadIdx.x; e < TC * N; e += BLK) s_y[e] = Y[(size_t)t0 * N + e];
  __syncthreads();
}

// ---- VALU: 8 lanes per filter ----
__global__ __launch_bounds__(BLK, 2) void stats_valu(const double* __restrict__ Y, double* __restrict__ out) {
  constexpr int L = 8;
  __shared__ double s_y[TC * N];
  __shared__ double2 s_mr[N];
  for (int i = threadIdx.x; i < N; i += BLK) s_mr[i] = make_double2(i + 1.0, 1.0 / (i + 1.0));
  const int j = threadIdx.x % L;
  const int b = blockIdx.x * (BLK / L) + threadIdx.x / L;
  double chk[NSTAT] = {};
  for (int t = 0; t < T; ++t) {
    if (t % TC == 0) stage(Y, s_y, t);
    const double* col = s_y + (t % TC) * N;
    double beta[4];
    filter_consts(b, t, beta);
    const double lam = 1e-2 + exp(beta[3]);
    const double rl = 1.0 / lam, dl = lam - 1e-2;
    const double c2 = beta[2] * dl, k1 = (beta[1] + beta[2]) * dl * rl;
    const double wj = exp(-lam * L);
    double z = exp(-lam * (j + 1));
    double s[NSTAT] = {};
#pragma unroll 2
    for (int i = j; i < N; i += L) {
      const double2 mr = s_mr[i];
      const double y = col[i];
      const double it = rl * mr.y;
      const double z2 = (1.0 - z) * it;
      const double z3 = z2 - z;
      const double z4 = z * fma(c2, mr.x, fma(-k1, it, k1));
      s[1] += z2;
      s[2] += z3;
      s[3] += z4;
      s[4] = fma(z2, z2, s[4]);
      s[5] = fma(z2, z3, s[5]);
      s[6] = fma(z2, z4, s[6]);
      s[7] = fma(z3, z3, s[7]);
      s[8] = fma(z3, z4, s[8]);
      s[9] = fma(z4, z4, s[9]);
      const double v = y - fma(beta[2], z3, fma(beta[1], z2, beta[0]));
      s[10] += v;
      s[11] = fma(z2, v, s[11]);
      s[12] = fma(z3, v, s[12]);
      s[13] = fma(z4, v, s[13]);
      s[14] = fma(v, v, s[14]);
      z *= wj;
    }
#pragma unroll
    for (int k = 1; k < NSTAT; ++k) {
      const double r = lvl_sum<2>(lvl_sum<1>(lvl_sum<0>(s[k])));
      chk[k] = fma(r, 1.0 + 1e-3 * (t & 7), chk[k]);  // keep every step's statistics live
    }
  }
  if (j == 0)
    for (int k = 1; k < NSTAT; ++k) out[(size_t)b * NSTAT + k] = chk[k];
}

// ---- MFMA: 16 lanes (one 4x4x4 block) per filter ----
__global__ __launch_bounds__(BLK, 2) void stats_mfma(const double* __restrict__ Y, double* __restrict__ out) {
  __shared__ double s_y[TC * N];
  __shared__ double2 s_mr[N];
  for (int i = threadIdx.x; i < N; i += BLK) s_mr[i] = make_double2(i + 1.0, 1.0 / (i + 1.0));
  const int lane = threadIdx.x & 63;
  const int k = lane >> 4;          // maturity slot within a chunk of 4
  const int blk = (lane >> 2) & 3;  // filter within the wave
  const int x = lane & 3;           // column: 0 → (A = 1, B = v), 1 → z2, 2 → z3, 3 → z4
  const int b = blockIdx.x * (BLK / 16) + (threadIdx.x >> 6) * 4 + blk;
  double chk = 0.0, chk_vv = 0.0;
  for (int t = 0; t < T; ++t) {
    if (t % TC == 0) stage(Y, s_y, t);
    const double* col = s_y + (t % TC) * N;
    double beta[4];
    filter_consts(b, t, beta);
    const double lam = 1e-2 + exp(beta[3]);
    const double rl = 1.0 / lam, dl = lam - 1e-2;
    const double c2 = beta[2] * dl, k1 = (beta[1] + beta[2]) * dl * rl;
    const double s12 = (beta[1] + beta[2]) * rl;
    // column value = z·(ca + cb/m + cc·m) + cd/m + ce + cf·y
    const double ca = x == 0 ? beta[2] : x == 1 ? 0.0 : x == 2 ? -1.0 : k1;
    const double cb = x == 0 ? s12 : x == 3 ? -k1 * rl : -rl;
    const double cc = x == 3 ? c2 : 0.0;
    const double cd = x == 0 ? -s12 : x == 3 ? 0.0 : rl;
    const double ce = x == 0 ? -beta[0] : 0.0;
    const double cf = x == 0 ? 1.0 : 0.0;
    const double w4 = exp(-lam * 4.0);
    double z = exp(-lam * (k + 1));
    typedef double d1;
    d1 acc0 = 0.0, acc1 = 0.0;
    double vv = 0.0;
#pragma unroll 2
    for (int c = 0; c < N / 4; ++c) {
      const double2 mr = s_mr[4 * c + k];
      const double y = col[4 * c + k];
      const double g = fma(cc, mr.x, fma(cb, mr.y, ca));
      const double val = fma(z, g, fma(cd, mr.y, fma(cf, y, ce)));
      const double a = x == 0 ? 1.0 : val;
      vv = fma(val, val, vv);
      if (c & 1)
        acc1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, val, acc1, 0, 0, 0);
      else
        acc0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, val, acc0, 0, 0, 0);
      z *= w4;
    }
    const double d = acc0 + acc1;  // lane 16i + 4blk + j holds D[i][j]
    // v'v: lanes x = 0 of the four maturity slots
    double r = vv + __shfl_xor(vv, 16);
    r = r + __shfl_xor(r, 32);
    const double wt = 1.0 + 1e-3 * (t & 7);
    chk = fma(d, wt, chk);
    chk_vv = fma(r, wt, chk_vv);
  }
  // D[i][j] for i = 0..3 (A: 1 z2 z3 z4), j = 0..3 (B: v z2 z3 z4)
  const int i = lane >> 4, jj = lane & 3;
  const int map[4][4] = {{10, 1, 2, 3}, {11, 4, 5, 6}, {12, 5, 7, 8}, {13, 6, 8, 9}};
  if (!(i == 2 && jj == 1) && !(i == 3 && jj <= 2 && jj >= 1)) out[(size_t)b * NSTAT + map[i][jj]] = chk;
  if (lane == 4 * blk) out[(size_t)b * NSTAT + 14] = chk_vv;
}

int main() {
  std::vector<double> hY((size_t)N * T);
  for (int t = 0; t < T; ++t)
    for (int i = 0; i < N; ++i) hY[(size_t)t * N + i] = 5.0 - 1.5 * exp(-0.06 * (i + 1)) + 0.3 * sin(0.01 * t * (i % 7 + 1));
  double *dY, *o1, *o2;
  (void)hipMalloc(&dY, sizeof(double) * hY.size());
  (void)hipMalloc(&o1, sizeof(double) * B * NSTAT);
  (void)hipMalloc(&o2, sizeof(double) * B * NSTAT);
  (void)hipMemcpy(dY, hY.data(), sizeof(double) * hY.size(), hipMemcpyHostToDevice);
  (void)hipMemset(o1, 0, sizeof(double) * B * NSTAT);
  (void)hipMemset(o2, 0, sizeof(double) * B * NSTAT);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best_v = 1e30f, best_m = 1e30f;
  for (int rep = 0; rep < 6; ++rep) {
    float ms;
    (void)hipEventRecord(e0);
    stats_valu<<<B / (BLK / 8), BLK>>>(dY, o1);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep) best_v = std::min(best_v, ms);
    (void)hipEventRecord(e0);
    stats_mfma<<<B / (BLK / 16), BLK>>>(dY, o2);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep) best_m = std::min(best_m, ms);
  }
  std::vector<double> h1((size_t)B * NSTAT), h2((size_t)B * NSTAT);
  (void)hipMemcpy(h1.data(), o1, sizeof(double) * h1.size(), hipMemcpyDeviceToHost);
  (void)hipMemcpy(h2.data(), o2, sizeof(double) * h2.size(), hipMemcpyDeviceToHost);
  double maxrel = 0.0;
  for (size_t q = 0; q < h1.size(); ++q) {
    if (q % NSTAT == 0) continue;
    const double den = std::fabs(h1[q]) > 1e-300 ? std::fabs(h1[q]) : 1.0;
    maxrel = std::max(maxrel, std::fabs(h1[q] - h2[q]) / den);
  }
  printf("statistics phase, N=%d T=%d B=%d: VALU (8 lanes/filter) %.3f ms, MFMA 4x4x4 (16 lanes/filter) %.3f ms, "
         "max rel diff %.2e\n", N, T, B, best_v, best_m, maxrel);
  return 0;
}

// steady_step_probe.hip — cycles per frozen-covariance steady step of the DNS filter in isolation (one wave per
// SIMD, 16 steps unrolled per block, operands read from LDS as the kernel reads them), in two forms:
//   V = 0  the kernel's form (yfm_fixedz.hpp collapsed_mean + propagate_mean_f): c = ĉ − β, x = S⁻¹c (cached
//          LDLᵀ), q = rr/σ² + c'x, β_{t|t} = β + P x, β ← δ + Φ β_{t|t} — a β→β chain ≈ 12 FP64 operations deep;
//   V = 1  the time-invariant form: β ← d + A β + B z̃ + b ȳ with A = Φ(I − P S⁻¹), B, b, d folded once at the
//          freeze; x = S⁻¹c only feeds q (off the chain) — the β→β chain is 3 FMAs deep.
// Same FP64 instruction count to within a few; if V = 1 runs much faster, the steady step is latency-bound.
// Build: hipcc --offload-arch=gfx950 -O3 tools/steady_step_probe.hip -o tools/steady_step_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int M = 3, TB = 16, NB = 37;  // 37 blocks of 16 = 592 steady steps (config 2: 583)

template <int V>
__global__ __launch_bounds__(256, 1) void probe(const double* __restrict__ init, double* __restrict__ out,
                                                 long long* __restrict__ cyc) {
  __shared__ double zs[4][TB][64][4];  // per wave: step × lane × (z̃1, z̃2, ȳ, ỹ'ỹ)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.x * 256 + threadIdx.x;
  for (int t = 0; t < TB; ++t)
#pragma unroll
    for (int k = 0; k < 4; ++k) zs[wave][t][lane][k] = init[(b * 7 + t * 4 + k) & 1023] * 1e-3;
  // a frozen state: P, R SPD, S = P + R factorised; Φ stable
  double P[M][M], R[M][M], Phi[M][M], delta[M], beta[M], L[M][M], rd[M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const double e = init[(b + 3 * i + j) & 1023] * 1e-2;
      P[i][j] = (i == j ? 0.5 : 0.0) + e * e;
      R[i][j] = (i == j ? 0.2 : 0.0) + 0.5 * e * e;
      Phi[i][j] = (i == j ? 0.9 : 0.01 * e);
      L[i][j] = 0.1 * e;
    }
    delta[i] = 0.01 * init[(b + i) & 1023];
    beta[i] = init[(b + 11 * i) & 1023];
    rd[i] = 1.0 / (0.7 + 0.01 * i);
  }
  const double rsig2 = 1.0 / (0.01 + 1e-4 * init[b & 1023]);
  // V = 1: A = Φ(I − P S⁻¹) ≈ any 3×3, B (3×2), bb (3), d (3) — values do not matter for timing
  double A[M][M], Bz[M][2], bb[M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
#pragma unroll
    for (int j = 0; j < M; ++j) A[i][j] = 0.5 * Phi[i][j] - 0.1 * P[i][j];
    Bz[i][0] = 0.1 * R[i][1];
    Bz[i][1] = 0.1 * R[i][2];
    bb[i] = 0.2 * Phi[i][0];
  }
  __syncthreads();
  double sumq = 0.0;
  long long csteady = 0;
  const long long c0 = __builtin_readcyclecounter();
  for (int blk = 0; blk < NB; ++blk) {
    // a new block of operands per block (the kernel's MFMA block writes them): not loop-invariant
    {
      const double pert = 1e-9 * blk;
#pragma unroll
      for (int t = 0; t < TB; ++t) {
        double2* q = reinterpret_cast<double2*>(&zs[wave][t][lane][0]);
        double2 v = q[0];
        v.x += pert;
        q[0] = v;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
    const long long cs = __builtin_readcyclecounter();
#pragma unroll
    for (int t = 0; t < TB; ++t) {
      const double2 z = *reinterpret_cast<const double2*>(&zs[wave][t][lane][0]);
      const double2 yb = *reinterpret_cast<const double2*>(&zs[wave][t][lane][2]);
      const double zt[2] = {z.x, z.y};
      // ĉ = R/σ²·(0, z̃), rr = ỹ'ỹ − z̃'ĉ, ĉ₀ += ȳ
      double zsc[2] = {zt[0] * rsig2, zt[1] * rsig2}, ch[M];
#pragma unroll
      for (int i = 0; i < M; ++i) ch[i] = fma(R[i][2], zsc[1], R[i][1] * zsc[0]);
      double rr = fma(-zt[1], ch[2], fma(-zt[0], ch[1], yb.y));
      ch[0] += yb.x;
      double c[M], x[M];
#pragma unroll
      for (int i = 0; i < M; ++i) x[i] = c[i] = ch[i] - beta[i];
      // x = S⁻¹c with the cached LDLᵀ
#pragma unroll
      for (int i = 0; i < M; ++i)
#pragma unroll
        for (int k = 0; k < i; ++k) x[i] = fma(-L[i][k], x[k], x[i]);
#pragma unroll
      for (int i = 0; i < M; ++i) x[i] *= rd[i];
#pragma unroll
      for (int i = M - 1; i >= 0; --i)
#pragma unroll
        for (int k = i + 1; k < M; ++k) x[i] = fma(-L[k][i], x[k], x[i]);
      double cx = 0.0;
#pragma unroll
      for (int i = 0; i < M; ++i) cx = fma(c[i], x[i], cx);
      sumq += fma(rr, rsig2, cx);
      if constexpr (V == 0) {
        double bf[M];
#pragma unroll
        for (int i = 0; i < M; ++i) {
          double s = beta[i];
#pragma unroll
          for (int k = 0; k < M; ++k) s = fma(P[i][k], x[k], s);
          bf[i] = s;
        }
#pragma unroll
        for (int i = 0; i < M; ++i) {
          double s = delta[i];
#pragma unroll
          for (int k = 0; k < M; ++k) s = fma(Phi[i][k], bf[k], s);
          beta[i] = s;
        }
      } else {
        double nb[M];
#pragma unroll
        for (int i = 0; i < M; ++i) {
          double s = fma(bb[i], yb.x, fma(Bz[i][1], zt[1], fma(Bz[i][0], zt[0], delta[i])));  // off the chain
#pragma unroll
          for (int k = 0; k < M; ++k) s = fma(A[i][k], beta[k], s);
          nb[i] = s;
        }
#pragma unroll
        for (int i = 0; i < M; ++i) beta[i] = nb[i];
      }
    }
#pragma unroll
    for (int i = 0; i < M; ++i) asm volatile("" ::"v"(beta[i]));
    asm volatile("" ::"v"(sumq));
    csteady += __builtin_readcyclecounter() - cs;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
  }
  const long long c1 = __builtin_readcyclecounter();
  out[b] = sumq + beta[0] + beta[1] + beta[2];
  if (lane == 0) {
    cyc[2 * (b >> 6)] = c1 - c0;
    cyc[2 * (b >> 6) + 1] = csteady;
  }
}

template <int V>
static void run(const double* d_init, double* d_out, long long* d_cyc, int B) {
  const int waves = B / 64;
  probe<V><<<B / 256, 256>>>(d_init, d_out, d_cyc);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    float ms;
    hipEventRecord(e0);
    probe<V><<<B / 256, 256>>>(d_init, d_out, d_cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  long long* h = new long long[2 * waves];
  hipMemcpy(h, d_cyc, sizeof(long long) * 2 * waves, hipMemcpyDeviceToHost);
  double mean = 0, mst = 0;
  for (int w = 0; w < waves; ++w) {
    mean += h[2 * w];
    mst += h[2 * w + 1];
  }
  mean /= waves;
  mst /= waves;
  printf("V=%d (%s): %.4f ms; s_memtime ticks per step: whole loop %.1f, steady steps only %.1f (%d steps)\n", V,
         V == 0 ? "kernel form, chain ~12 deep" : "time-invariant form, chain 3 deep", best, mean / (NB * TB),
         mst / (NB * TB), NB * TB);
  delete[] h;
}

int main() {
  const int B = 65536;
  double *d_init, *d_out;
  long long* d_cyc;
  hipMalloc(&d_init, 1024 * 8);
  hipMalloc(&d_out, B * 8);
  hipMalloc(&d_cyc, (B / 64) * 16);
  double h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = 0.5 + 0.001 * ((i * 7919) % 997);
  hipMemcpy(d_init, h, sizeof h, hipMemcpyHostToDevice);
  for (int k = 0; k < 20; ++k) probe<0><<<B / 256, 256>>>(d_init, d_out, d_cyc);  // clock ramp
  hipDeviceSynchronize();
  run<0>(d_init, d_out, d_cyc, B);
  run<1>(d_init, d_out, d_cyc, B);
  run<0>(d_init, d_out, d_cyc, B);
  run<1>(d_init, d_out, d_cyc, B);
  return 0;
}

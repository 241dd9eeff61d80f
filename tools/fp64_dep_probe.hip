// fp64_dep_probe.hip — how far apart dependent FP64 VALU instructions can issue at ONE wave per SIMD (the
// occupancy of the certified TVλ and DNS kernels): v_fma_f64 / v_add_f64 chains, 1, 2, 3, 4 and 8 independent
// chains interleaved, straight-line (inner loop unrolled 8×).  Cycles per instruction = 1,024 SIMDs × instructions ÷
// (time × clock); the clock is reported by s_memtime / s_memrealtime inside the kernel.  Also the σ-split
// accumulation of yfm_dd.hpp (dd_acc::add_prod_sx) as one dependent 5-instruction chain per product, with 1, 2 and 4
// products interleaved.  Build: hipcc --offload-arch=gfx950 -O3 tools/fp64_dep_probe.hip -o tools/fp64_dep_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang diagnostic ignored "-Wunused-result"

template <int CH, bool ADD>
__global__ __launch_bounds__(256) void chains(double* out, int iters, double a, double b, long long* clk) {
  double acc[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) acc[i] = threadIdx.x * 1e-3 + i;
  const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int i = 0; i < CH; ++i) acc[i] = ADD ? acc[i] + a : fma(acc[i], a, b);
  }
  const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  double s = 0;
#pragma unroll
  for (int i = 0; i < CH; ++i) s += acc[i];
  if (s == 12345.678) out[0] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = r1 - r0;
  }
}

// σ-split product accumulation, as yfm_dd.hpp emits it: q = fma(a, b, σ) − σ; hi += q; r = fma(a, b, −q); lo += r
template <int P>
__global__ __launch_bounds__(256) void sx(double* out, int iters, double sg, long long* clk) {
  double hi[P], lo[P], x[P];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    hi[i] = 0.0;
    lo[i] = 0.0;
    x[i] = 1.0 + threadIdx.x * 1e-6 + i * 1e-3;
  }
  const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < P; ++i) {
        const double q = __builtin_fma(x[i], x[i], sg) - sg;
        hi[i] += q;
        lo[i] += __builtin_fma(x[i], x[i], -q);
        x[i] = x[i] * 0.9999999;  // a fresh product per step (one more dependent instruction)
      }
  }
  const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  double s = 0;
#pragma unroll
  for (int i = 0; i < P; ++i) s += hi[i] + lo[i];
  if (s == 12345.678) out[0] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = r1 - r0;
  }
}

template <typename K>
static void run(const char* name, K launch, double instr_per_iter_per_lane, double* d, long long* c) {
  const int iters = 4000, blocks = 256;  // one wave per SIMD
  launch(blocks, 10);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e30f;
  long long cl[2];
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    launch(blocks, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) {
      best = ms;
      hipMemcpy(cl, c, sizeof(cl), hipMemcpyDeviceToHost);
    }
  }
  const double instr = instr_per_iter_per_lane * iters;  // per wave
  const double cyc = (double)cl[0];                      // s_memtime cycles of wave 0's loop
  const double mhz = cl[1] > 0 ? 100.0 * (double)cl[0] / (double)cl[1] : 0.0;
  printf("%-40s %.2f cycles per instruction (in-kernel clock %.0f MHz; launch %.3f ms)\n", name, cyc / instr, mhz, best);
}

int main() {
  double* d;
  long long* c;
  hipMalloc(&d, 8);
  hipMalloc(&c, 16);
  for (int k = 0; k < 4; ++k) chains<16, false><<<256 * 8, 256>>>(d, 20000, 0.999999, 1e-7, c);  // clock ramp
  hipDeviceSynchronize();
#define RUN_CH(N, ADD, NAME) \
  run(NAME, [&](int b, int it) { chains<N, ADD><<<b, 256>>>(d, it, 0.999999, 1e-7, c); }, 8.0 * N, d, c)
  RUN_CH(1, false, "v_fma_f64, 1 chain");
  RUN_CH(2, false, "v_fma_f64, 2 chains");
  RUN_CH(3, false, "v_fma_f64, 3 chains");
  RUN_CH(4, false, "v_fma_f64, 4 chains");
  RUN_CH(8, false, "v_fma_f64, 8 chains");
  RUN_CH(1, true, "v_add_f64, 1 chain");
  RUN_CH(2, true, "v_add_f64, 2 chains");
  RUN_CH(4, true, "v_add_f64, 4 chains");
#define RUN_SX(N) run("sigma-split product, " #N " interleaved", [&](int b, int it) { sx<N><<<b, 256>>>(d, it, 0x1p10, c); }, 4.0 * 6 * N, d, c)
  RUN_SX(1);
  RUN_SX(2);
  RUN_SX(4);
  RUN_SX(8);
  return 0;
}

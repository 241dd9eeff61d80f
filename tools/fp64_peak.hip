// fp64_peak.hip — measure the sustained v_fma_f64 rate of this MI355X (the local
// guide lists no FP64 figure; the roofline peak in bench.py is the AMD spec, and
// this diagnostic checks it).  Build: hipcc --offload-arch=gfx950 -O3 fp64_peak.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int ACC>
__global__ __launch_bounds__(256) void fma_loop(double* out, int iters, double a, double b) {
  double acc[ACC];
#pragma unroll
  for (int i = 0; i < ACC; ++i) acc[i] = threadIdx.x * 1e-3 + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) acc[i] = fma(acc[i], a, b);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < ACC; ++i) s += acc[i];
  if (s == 12345.678) out[0] = s;  // keep the work live
}

template <int ACC>
static void run(int blocks_per_cu, const char* tag) {
  double* d;
  hipMalloc(&d, 8);
  const int iters = 20000, blocks = 256 * blocks_per_cu;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  fma_loop<ACC><<<blocks, 256>>>(d, 100, 0.999999, 1e-7);
  hipEventRecord(e0);
  fma_loop<ACC><<<blocks, 256>>>(d, iters, 0.999999, 1e-7);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * ACC * (double)iters * blocks * 256;
  printf("%-28s ACC=%2d blocks/CU=%d  %.2f TFLOP/s\n", tag, ACC, blocks_per_cu, flops / (ms * 1e-3) / 1e12);
  hipFree(d);
}

int main() {
  run<16>(1, "1 wave/SIMD");
  run<8>(1, "1 wave/SIMD");
  run<4>(1, "1 wave/SIMD");
  run<16>(2, "2 waves/SIMD");
  run<16>(8, "8 waves/SIMD");
  return 0;
}

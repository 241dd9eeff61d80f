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
  float ms = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {  // best of 5 (clocks settle after the ramp in main)
    float m;
    hipEventRecord(e0);
    fma_loop<ACC><<<blocks, 256>>>(d, iters, 0.999999, 1e-7);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&m, e0, e1);
    if (m < ms) ms = m;
  }
  const double flops = 2.0 * ACC * (double)iters * blocks * 256;
  printf("%-28s ACC=%2d blocks/CU=%d  %.2f TFLOP/s\n", tag, ACC, blocks_per_cu, flops / (ms * 1e-3) / 1e12);
  hipFree(d);
}

int main() {
  {  // ≈0.2 s of full-chip FMA work first, so the card is at its steady clock when timed
    double* d;
    hipMalloc(&d, 8);
    for (int k = 0; k < 4; ++k) fma_loop<16><<<256 * 8, 256>>>(d, 200000, 0.999999, 1e-7);
    hipDeviceSynchronize();
    hipFree(d);
  }
  run<16>(1, "1 wave/SIMD");
  run<8>(1, "1 wave/SIMD");
  run<4>(1, "1 wave/SIMD");
  run<16>(2, "2 waves/SIMD");
  run<16>(8, "8 waves/SIMD");
  return 0;
}

// fp64_waves.hip — sustained v_fma_f64 rate against waves per SIMD and independent chains per wave,
// straight-line (the inner loop unrolled 8×, so loop control is < 2% of the issue slots).  Decides whether a
// register-light DNS design (several waves per SIMD) could exceed the one-wave rate the 490-register kernel
// runs at.  Build: hipcc --offload-arch=gfx950 -O3 tools/fp64_waves.hip -o tools/fp64_waves
#include <hip/hip_runtime.h>
#include <cstdio>

template <int ACC>
__global__ __launch_bounds__(256) void fma_chains(double* out, int iters, double a, double b) {
  double acc[ACC];
#pragma unroll
  for (int i = 0; i < ACC; ++i) acc[i] = threadIdx.x * 1e-3 + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int i = 0; i < ACC; ++i) acc[i] = fma(acc[i], a, b);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < ACC; ++i) s += acc[i];
  if (s == 12345.678) out[0] = s;
}

template <int ACC>
static void run(int waves_per_simd) {
  double* d;
  hipMalloc(&d, 8);
  const int iters = 2000, blocks = 256 * waves_per_simd;  // 256 CUs, 4 waves (one per SIMD) per block
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  fma_chains<ACC><<<blocks, 256>>>(d, 10, 0.999999, 1e-7);
  float ms = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    float m;
    hipEventRecord(e0);
    fma_chains<ACC><<<blocks, 256>>>(d, iters, 0.999999, 1e-7);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&m, e0, e1);
    if (m < ms) ms = m;
  }
  const double flops = 2.0 * ACC * 8.0 * (double)iters * blocks * 256;
  printf("waves/SIMD %d  chains %2d  %.2f TFLOP/s\n", waves_per_simd, ACC, flops / (ms * 1e-3) / 1e12);
  hipFree(d);
}

int main() {
  double* d;
  hipMalloc(&d, 8);
  for (int k = 0; k < 4; ++k) fma_chains<16><<<256 * 8, 256>>>(d, 20000, 0.999999, 1e-7);  // clock ramp
  hipDeviceSynchronize();
  hipFuncAttributes fa;
  hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&fma_chains<32>));
  printf("fma_chains<32>: %d VGPRs (numRegs)\n", fa.numRegs);
  for (int w : {1, 2, 3, 4, 8}) {
    run<4>(w);
    run<8>(w);
    run<16>(w);
    run<32>(w);
  }
  return 0;
}

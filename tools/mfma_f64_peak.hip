// mfma_f64_peak.hip — sustained rate of v_mfma_f64_16x16x4_f64 on this MI355X, to price the
// MFMA formulation of the TVλ per-step statistics: each instruction does
// 16·16·4·2 = 2,048 flops; the per-filter Gram [1 z2 z3 z4 v]'[1 z2 z3 z4 v] only uses the
// block-diagonal part of the 16×16 product (3 filters × 5×5 = 75 of 256 outputs), so the
// useful rate of that mapping is this peak × 75/256.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_f64_peak.hip -o mfma_f64_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int ACC>
__global__ __launch_bounds__(256) void mfma_loop(double* out, int iters, double a, double b) {
  d4 acc[ACC];
#pragma unroll
  for (int i = 0; i < ACC; ++i) acc[i] = d4{threadIdx.x * 1e-3, 1.0 * i, 0.5, 0.25};
  double x = a + threadIdx.x * 1e-9, y = b;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[i], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < ACC; ++i) s += acc[i].x + acc[i].y + acc[i].z + acc[i].w;
  if (s == 12345.678) out[0] = s;  // keep the work live
}

template <int ACC>
static void run(int blocks_per_cu, const char* tag) {
  double* d;
  (void)hipMalloc(&d, 8);
  const int iters = 20000, blocks = 256 * blocks_per_cu;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  mfma_loop<ACC><<<blocks, 256>>>(d, 100, 1e-6, 1e-7);
  float ms = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    float m;
    (void)hipEventRecord(e0);
    mfma_loop<ACC><<<blocks, 256>>>(d, iters, 1e-6, 1e-7);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&m, e0, e1);
    if (m < ms) ms = m;
  }
  // per wave and instruction: 16·16·4 multiply-adds
  const double flops = 2048.0 * ACC * (double)iters * blocks * 4;
  const double tf = flops / (ms * 1e-3) / 1e12;
  printf("%-14s ACC=%d blocks/CU=%d  %.2f TFLOP/s  (%.1f TF useful at 75/256)\n", tag, ACC, blocks_per_cu, tf,
         tf * 75.0 / 256.0);
  (void)hipFree(d);
}

int main() {
  {
    double* d;
    (void)hipMalloc(&d, 8);
    for (int k = 0; k < 4; ++k) mfma_loop<4><<<256 * 8, 256>>>(d, 100000, 1e-6, 1e-7);
    (void)hipDeviceSynchronize();
    (void)hipFree(d);
  }
  run<4>(1, "1 wave/SIMD");
  run<8>(1, "1 wave/SIMD");
  run<4>(2, "2 waves/SIMD");
  run<4>(4, "4 waves/SIMD");
  return 0;
}

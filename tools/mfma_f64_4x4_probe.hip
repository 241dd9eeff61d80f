// mfma_f64_4x4_probe.hip — operand layout and sustained rate of v_mfma_f64_4x4x4_4b_f64
// (four independent 4×4×4 FP64 products per wave), to price an MFMA formulation of the TVλ
// per-step Gram: one block = one filter's [4 loading columns × 4 maturities]
// slice, D = Wᵀ W accumulated over the maturities, every output element useful.
//
// Layout probe: A = 2^lane, B = one-hot at lane q.  Then D[l] is the A element paired with
// B's lane q at output position l, so for every q we print (q → the lanes l with D ≠ 0 and the
// A lane that multiplied it).  Rate: independent accumulator chains at 1/2/4 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_f64_4x4_probe.hip -o mfma_f64_4x4_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

__global__ void probe(double* out, int q) {
  const int l = threadIdx.x;
  const double a = ldexp(1.0, l);
  const double b = (l == q) ? 1.0 : 0.0;
  double c = 0.0;
  c = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
  out[l] = c;
}

template <int ACC>
__global__ __launch_bounds__(256) void rate_loop(double* out, int iters, double a, double b) {
  double acc[ACC];
#pragma unroll
  for (int i = 0; i < ACC; ++i) acc[i] = threadIdx.x * 1e-3 + i;
  const double x = a + threadIdx.x * 1e-9, y = b;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, acc[i], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < ACC; ++i) s += acc[i];
  if (s == 12345.678) out[0] = s;
}

template <int ACC>
static void rate(int blocks_per_cu, const char* tag) {
  double* d;
  (void)hipMalloc(&d, 8);
  const int iters = 40000, blocks = 256 * blocks_per_cu;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  rate_loop<ACC><<<blocks, 256>>>(d, 100, 1e-6, 1e-7);
  float ms = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    float m;
    (void)hipEventRecord(e0);
    rate_loop<ACC><<<blocks, 256>>>(d, iters, 1e-6, 1e-7);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&m, e0, e1);
    if (m < ms) ms = m;
  }
  // per wave and instruction: 4 blocks × 4·4·4 multiply-adds = 512 flops
  const double insts = (double)ACC * iters * blocks * 4;
  const double tf = 512.0 * insts / (ms * 1e-3) / 1e12;
  const double cyc = (ms * 1e-3) * 2.4e9 / ((double)ACC * iters * blocks_per_cu);  // per inst per SIMD
  printf("%-14s ACC=%d  %.2f TFLOP/s  (%.1f SIMD cycles per instruction at 2.4 GHz)\n", tag, ACC, tf, cyc);
  (void)hipFree(d);
}

int main() {
  double *d, h[64];
  (void)hipMalloc(&d, 64 * sizeof(double));
  for (int q = 0; q < 64; ++q) {
    probe<<<1, 64>>>(d, q);
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("B lane %2d:", q);
    for (int l = 0; l < 64; ++l)
      if (h[l] != 0.0) printf(" D%d<-A%d", l, (int)std::lround(std::log2(h[l])));
    printf("\n");
  }
  (void)hipFree(d);
  {
    double* w;
    (void)hipMalloc(&w, 8);
    for (int k = 0; k < 4; ++k) rate_loop<8><<<256 * 8, 256>>>(w, 100000, 1e-6, 1e-7);
    (void)hipDeviceSynchronize();
    (void)hipFree(w);
  }
  rate<4>(1, "1 wave/SIMD");
  rate<8>(1, "1 wave/SIMD");
  rate<16>(1, "1 wave/SIMD");
  rate<8>(2, "2 waves/SIMD");
  rate<8>(4, "4 waves/SIMD");
  return 0;
}

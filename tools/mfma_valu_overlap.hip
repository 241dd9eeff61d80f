// mfma_valu_overlap.hip — do FP64 MFMA and FP64 VALU work overlap on one MI355X SIMD?
// (the DNS steady block is Z'ỹ MFMAs + a VALU mean update, issued in order by one wave.)
// Workgroups of 512 threads = 8 waves, two per SIMD.  Per wave: `im` MFMA iterations (ACC independent
// v_mfma_f64_16x16x4 or 4x4x4_4b accumulators) and/or `iv` VALU iterations (8 independent v_fma_f64 chains).
//   mode 0: every wave MFMA only          mode 1: every wave VALU only
//   mode 2: waves 0-3 MFMA, waves 4-7 VALU (each SIMD one of each: cross-wave overlap)
//   mode 3: one wave per SIMD (256 threads) doing MFMA and VALU interleaved in one stream
//   mode 4: one wave per SIMD, MFMA only      mode 5: one wave per SIMD, VALU only
// Build: hipcc --offload-arch=gfx950 -O3 mfma_valu_overlap.hip -o mfma_valu_overlap
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <bool BIG>
__device__ __forceinline__ void mfma_part(double x, double y, d4 (&acc)[4], double (&a1)[16]) {
  if constexpr (BIG) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[i], 0, 0, 0);
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) a1[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, a1[i], 0, 0, 0);
  }
}

__device__ __forceinline__ void valu_part(double (&v)[8], double a, double b) {
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = __builtin_fma(v[i], a, b);
}

template <bool BIG>
__global__ __launch_bounds__(512) void overlap(double* out, int mode, int im, int iv, double a, double b) {
  const int wave = threadIdx.x >> 6;
  d4 acc[4];
  double a1[16];
  double v[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = d4{threadIdx.x * 1e-3, 1.0 * i, 0.5, 0.25};
#pragma unroll
  for (int i = 0; i < 16; ++i) a1[i] = threadIdx.x * 1e-3 + i;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = threadIdx.x * 1e-6 + i;
  const double x = a + threadIdx.x * 1e-9, y = b;
  bool do_m = false, do_v = false, inter = false;
  if (mode == 0 || mode == 4) do_m = true;
  if (mode == 1 || mode == 5) do_v = true;
  if (mode == 2) {
    do_m = wave < 4;
    do_v = wave >= 4;
  }
  if (mode == 3) inter = true;
  if (inter) {
    const int n = im > iv ? im : iv;
    for (int it = 0; it < n; ++it) {
      if (it < im) mfma_part<BIG>(x, y, acc, a1);
      if (it < iv) valu_part(v, a, b);
    }
  } else {
    if (do_m)
      for (int it = 0; it < im; ++it) mfma_part<BIG>(x, y, acc, a1);
    if (do_v)
      for (int it = 0; it < iv; ++it) valu_part(v, a, b);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) s += acc[i].x + acc[i].y + acc[i].z + acc[i].w;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += a1[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) s += v[i];
  if (s == 12345.678) out[0] = s;  // keep the work live
}

template <bool BIG>
static float run(int mode, int im, int iv) {
  double* d;
  (void)hipMalloc(&d, 8);
  const int threads = (mode >= 3) ? 256 : 512;
  const int blocks = 256;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  overlap<BIG><<<blocks, threads>>>(d, mode, 10, 10, 1e-6, 1e-7);
  float ms = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    float m;
    (void)hipEventRecord(e0);
    overlap<BIG><<<blocks, threads>>>(d, mode, im, iv, 1e-6, 1e-7);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&m, e0, e1);
    if (m < ms) ms = m;
  }
  (void)hipFree(d);
  return ms;
}

int main() {
  {  // clock settle
    double* d;
    (void)hipMalloc(&d, 8);
    for (int k = 0; k < 4; ++k) overlap<true><<<256 * 4, 512>>>(d, 0, 20000, 0, 1e-6, 1e-7);
    (void)hipDeviceSynchronize();
    (void)hipFree(d);
  }
  const int im = 20000;
  for (int big = 1; big >= 0; --big) {
    auto R = [&](int mode, int a, int b) { return big ? run<true>(mode, a, b) : run<false>(mode, a, b); };
    // the VALU count that matches the MFMA time of one wave per SIMD
    const float tm = R(4, im, 0);
    const float tv1 = R(5, 0, im);
    const int iv = (int)(im * (tm / tv1));
    const float tv = R(5, 0, iv);
    printf("%s: 1 wave/SIMD MFMA-only %d iters %.3f ms; VALU-only %d iters (32 fma each) %.3f ms\n",
           big ? "16x16x4" : "4x4x4_4b", im, tm, iv, tv);
    printf("  mode 3 (one wave, interleaved): %.3f ms  (sum %.3f, max %.3f)\n", R(3, im, iv), tm + tv,
           tm > tv ? tm : tv);
    printf("  mode 0 (2 waves/SIMD, both MFMA): %.3f ms\n", R(0, im, 0));
    printf("  mode 1 (2 waves/SIMD, both VALU): %.3f ms\n", R(1, 0, iv));
    printf("  mode 2 (2 waves/SIMD, one MFMA + one VALU): %.3f ms\n", R(2, im, iv));
  }
  return 0;
}

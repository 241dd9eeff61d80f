// empty_launch_probe.hip — what an "empty" launch costs on the stream (the DNS path's deferral kernel runs after
// every loglik launch and usually finds its list empty: 4.6 µs in rocprofv3).  Kernels that read a zero count and
// return, launched back to back 2,000 times after a 50 µs busy kernel:
//   K0  no scratch, 64 VGPRs                 K1  the same body with a 4 KB private array (scratch per lane)
//   K2  no scratch, 256 VGPR + AGPR pressure  (occupancy-limited waves, like the dd kernel)
// Build: hipcc --offload-arch=gfx950 -O3 tools/empty_launch_probe.hip -o tools/empty_launch_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(256) void busy(double* x, int n) {
  double v = x[threadIdx.x];
  for (int i = 0; i < n; ++i) v = fma(v, 0.999999, 1e-9);
  x[blockIdx.x * 256 + threadIdx.x] = v;
}

__global__ __launch_bounds__(256) void k0(const int* __restrict__ count, double* __restrict__ out) {
  const int n = *count;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) out[i] = 1.0;
}

__global__ __launch_bounds__(256) void k1(const int* __restrict__ count, double* __restrict__ out) {
  const int n = *count;
  double priv[512];
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    for (int k = 0; k < 512; ++k) priv[k] = out[(i + k) % 4096];
    out[i] = priv[(i * 7) & 511];
  }
}

__global__ __launch_bounds__(256) void k2(const int* __restrict__ count, double* __restrict__ out) {
  const int n = *count;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    double a[200];
#pragma unroll
    for (int k = 0; k < 200; ++k) a[k] = out[(i + 37 * k) & 4095];
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int k = 0; k < 200; ++k) s = fma(a[k], a[(k + r) % 200], s);
    out[i] = s;
  }
}

template <typename F>
static void run(const char* name, F launch, double* x) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    busy<<<1024, 256>>>(x, 20000);
    (void)hipEventRecord(e0);
    for (int k = 0; k < 2000; ++k) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%s: %.2f us per launch\n", name, 1e3 * ms / 2000);
  }
}

int main() {
  int* d_count;
  double *d_out, *d_x;
  (void)hipMalloc(&d_count, sizeof(int));
  (void)hipMemset(d_count, 0, sizeof(int));
  (void)hipMalloc(&d_out, 4096 * 8);
  (void)hipMalloc(&d_x, 1024 * 256 * 8);
  (void)hipMemset(d_x, 0, 1024 * 256 * 8);
  run("K0 empty, no scratch, grid 256", [&] { k0<<<256, 256>>>(d_count, d_out); }, d_x);
  run("K1 empty, 4 KB scratch per lane, grid 256", [&] { k1<<<256, 256>>>(d_count, d_out); }, d_x);
  run("K1 empty, 4 KB scratch per lane, grid 8", [&] { k1<<<8, 256>>>(d_count, d_out); }, d_x);
  run("K2 empty, high register count, grid 256", [&] { k2<<<256, 256>>>(d_count, d_out); }, d_x);
  // alternating with a busy kernel (the loglik path's pattern): busy + empty vs busy alone
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[] = {"busy alone", "busy + K0", "busy + K1"};
  for (int v = 0; v < 3; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipEventRecord(e0);
      for (int k = 0; k < 200; ++k) {
        busy<<<1024, 256>>>(d_x, 2000);
        if (v == 1) k0<<<256, 256>>>(d_count, d_out);
        if (v == 2) k1<<<256, 256>>>(d_count, d_out);
      }
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("%s: %.2f us per step\n", names[v], 1e3 * ms / 200);
    }
  }
  return 0;
}

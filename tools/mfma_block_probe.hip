// mfma_block_probe.hip — cycles of the DNS Z'ỹ MFMA block in isolation (one wave per SIMD): 8 B operands
// read from LDS, 64 v_mfma_f64_16x16x4 (8 row tiles × 8 k-steps, two groups of 4 tiles), the D tiles stored
// to the wave's LDS scratch (σ layout: two 16-byte stores per tile), lgkmcnt(0) — as in
// yieldfactormodels.jl_amd/csrc/yfm_kernels.hip.  Variants:
//   V = 0  A fragments in VGPRs
//   V = 1  A fragments pinned in AGPRs (the kernel's allocation: the compiler copies them to VGPRs, or not)
//   V = 2  as 0 without the stores (the MFMA floor: 64 × 64 cycles = 4,096 per block at 32 FP64 flop/clk)
//   V = 3  as 0, stores issued but no lgkmcnt(0) wait at the block's end
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_block_probe.hip -o tools/mfma_block_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int NRT = 8, NK = 8, RGN = 4, SS = 130, NB = 38, LDP = 34;

template <int V>
__global__ __launch_bounds__(256, 1) void probe(const double* __restrict__ init, double* __restrict__ out,
                                                 long long* __restrict__ cyc) {
  __shared__ __attribute__((aligned(16))) double panel[64 * LDP];
  __shared__ __attribute__((aligned(16))) double scratch[4][16 * SS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 64 * LDP; i += 256) panel[i] = init[i & 1023];
  double Af[NRT][NK];
#pragma unroll
  for (int r = 0; r < NRT; ++r)
#pragma unroll
    for (int k = 0; k < NK; ++k) Af[r][k] = init[(lane * 13 + r * 7 + k) & 1023];
  __syncthreads();
  double* scr = scratch[wave];
  double sink = 0.0;
  long long tot = 0;
  for (int blk = 0; blk < NB; ++blk) {
    if constexpr (V == 1) {
#pragma unroll
      for (int r = 0; r < NRT; ++r)
#pragma unroll
        for (int k = 0; k < NK; ++k) asm volatile("" : "+a"(Af[r][k]));
    }
    const double* cb = panel + (blk & 3) * 16 * LDP;
    double bvk[NK];
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      const int m = 4 * kk + (lane >> 4);
      bvk[kk] = (m < 30) ? cb[(lane & 15) * LDP + m] : 0.0;
    }
    const long long c0 = __builtin_readcyclecounter();
#pragma unroll
    for (int r0 = 0; r0 < NRT; r0 += RGN) {
      d4 acc[RGN];
#pragma unroll
      for (int r = 0; r < RGN; ++r) acc[r] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < NK; ++kk)
#pragma unroll
        for (int r = 0; r < RGN; ++r)
          acc[r] = __builtin_amdgcn_mfma_f64_16x16x4f64(Af[r0 + r][kk], bvk[kk], acc[r], 0, 0, 0);
      if constexpr (V == 2) {
#pragma unroll
        for (int r = 0; r < RGN; ++r) asm volatile("" ::"a"(acc[r]));
      } else {
#pragma unroll
        for (int r = 0; r < RGN; ++r) {
          double* d = scr + (lane & 15) * SS + 16 * (r0 + r) + 4 * (lane >> 4);
          *reinterpret_cast<double2*>(d) = make_double2(acc[r][0], acc[r][1]);
          *reinterpret_cast<double2*>(d + 2) = make_double2(acc[r][2], acc[r][3]);
        }
      }
    }
    if constexpr (V != 3) __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    tot += __builtin_readcyclecounter() - c0;
    if constexpr (V == 3) __builtin_amdgcn_s_waitcnt(0xc07f);
    sink += scr[lane * 2 + (blk & 7)];
    __builtin_amdgcn_wave_barrier();
  }
  out[blockIdx.x * 256 + threadIdx.x] = sink;
  if (lane == 0) cyc[blockIdx.x * 4 + wave] = tot;
}

template <int V>
static void run(const double* d_init, double* d_out, long long* d_cyc, int nblk) {
  probe<V><<<nblk, 256>>>(d_init, d_out, d_cyc);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    float ms;
    hipEventRecord(e0);
    probe<V><<<nblk, 256>>>(d_init, d_out, d_cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  const int waves = nblk * 4;
  long long* h = new long long[waves];
  hipMemcpy(h, d_cyc, sizeof(long long) * waves, hipMemcpyDeviceToHost);
  double mean = 0;
  for (int w = 0; w < waves; ++w) mean += h[w];
  mean /= waves;
  const char* name[] = {"A in VGPRs", "A pinned in AGPRs", "no stores (MFMA floor)", "stores, no final wait"};
  printf("V=%d (%s): %.4f ms; s_memtime ticks per MFMA block %.1f\n", V, name[V], best, mean / NB);
  delete[] h;
}

int main() {
  const int nblk = 256;  // one workgroup per CU, one wave per SIMD
  double *d_init, *d_out;
  long long* d_cyc;
  hipMalloc(&d_init, 1024 * 8);
  hipMalloc(&d_out, nblk * 256 * 8);
  hipMalloc(&d_cyc, nblk * 4 * 8);
  double h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = 0.5 + 0.001 * ((i * 7919) % 997);
  hipMemcpy(d_init, h, sizeof h, hipMemcpyHostToDevice);
  for (int k = 0; k < 20; ++k) probe<0><<<nblk, 256>>>(d_init, d_out, d_cyc);
  hipDeviceSynchronize();
  for (int rep = 0; rep < 2; ++rep) {
    run<0>(d_init, d_out, d_cyc, nblk);
    run<1>(d_init, d_out, d_cyc, nblk);
    run<2>(d_init, d_out, d_cyc, nblk);
    run<3>(d_init, d_out, d_cyc, nblk);
  }
  return 0;
}

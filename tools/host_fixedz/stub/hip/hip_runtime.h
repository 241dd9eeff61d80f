// Host stand-in for <hip/hip_runtime.h>, ONLY for tools/host_fixedz/harness.cpp: it lets the per-lane
// filter code of csrc/yfm_fixedz.hpp / yfm_device.hpp compile for the CPU (one lane, no wave), so the
// C++ of the filter can run under MemorySanitizer.  Device-only intrinsics the harness never reaches are
// declared but not defined.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>

#define __device__
#define __host__
#define __global__
#define __forceinline__ inline __attribute__((always_inline))
#define __shared__
#define __launch_bounds__(...)

struct yfm_host_dim3 {
  unsigned x = 0, y = 0, z = 0;
};
static yfm_host_dim3 threadIdx, blockIdx, blockDim;
struct double2 {
  double x, y;
};
inline double2 make_double2(double a, double b) { return {a, b}; }
using std::exp;
using std::fabs;
using std::fma;
using std::fmax;
using std::fmin;
using std::isfinite;
using std::log;
using std::max;
using std::min;

// v_rcp_f64 is an approximation on the GPU; the host harness compares forms with each other, not bits
// with the GPU, so the exact reciprocal stands in for it
inline double __builtin_amdgcn_rcp(double d) { return 1.0 / d; }
inline int __builtin_amdgcn_frexp_exp(double m) {
  int e;
  (void)std::frexp(m, &e);
  return e;
}
inline double __builtin_amdgcn_frexp_mant(double m) {
  int e;
  return std::frexp(m, &e);
}
inline bool __all(bool x) { return x; }
inline bool __any(bool x) { return x; }
inline unsigned atomicAdd(unsigned* p, unsigned v) {
  const unsigned o = *p;
  *p += v;
  return o;
}
int __builtin_amdgcn_mov_dpp(int, int, int, int, bool);
int __double2loint(double);
int __double2hiint(double);
double __hiloint2double(int, int);
struct yfm_host_pair {
  int v[2];
  int operator[](int i) const { return v[i]; }
};
yfm_host_pair __builtin_amdgcn_permlane16_swap(int, int, bool, bool);
yfm_host_pair __builtin_amdgcn_permlane32_swap(int, int, bool, bool);
void __builtin_amdgcn_wave_barrier();
void __builtin_amdgcn_fence(int, const char*);

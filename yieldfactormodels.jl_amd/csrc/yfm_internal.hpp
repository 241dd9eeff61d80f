// yfm_internal.hpp — launch interface between the C ABI (yfm_capi.hip) and the kernels.
#pragma once
#include <hip/hip_runtime.h>

namespace yfm {

struct LaunchArgs {
  const double* theta;  // P×B device
  int P, B, space;
  const double* panel;  // prepared panel (T × ldp)
  const double* raw;    // caller's panel N×T column-major (device copy)
  int T, N, np, ldp;
  const double* mats;   // N device
  const int* T_use;     // B device or nullptr
  double* out;          // B device
  unsigned int* flags;  // 2 device counters
  double* rec_beta;     // optional trajectories
  double* rec_P;
  double* scratch;      // per-candidate work records (tvl_scratch_bytes)
  hipStream_t stream;
};

// padded maturity count NP the fixed-loading kernel is instantiated for (-1: none)
int fixedz_np_for(int N);
hipError_t launch_fixedz(int kind, const LaunchArgs& a);
// TVλ EKF kernel (yfm_tvl.hip): lanes per filter for a batch, largest N, launcher
int tvl_lanes_for(int B, int N);
int tvl_max_n();
size_t tvl_scratch_bytes(int B);
// Maturity jump table for the TVλ exp recurrence (built on the host per lane count L):
// the distinct values d_k of m_{i+L} − m_i and, per maturity i, the index k of its jump.
// K = 0 disables the recurrence (one exp per maturity).
constexpr int kTvlGaps = 8;
struct TvlGaps {
  int K = 0;
  const double* d = nullptr;  // device, kTvlGaps
  const int* idx = nullptr;   // device, N
};
hipError_t launch_tvl(const LaunchArgs& a, const TvlGaps& g, int lanes);
hipError_t launch_prep_panel(const double* Y, int N, int T, int np, int ldp, double* out, hipStream_t s);

}  // namespace yfm

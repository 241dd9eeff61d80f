// yfm_internal.hpp — launch interface between the C ABI (yfm_capi.hip) and the kernels.
#pragma once
#include <hip/hip_runtime.h>

namespace yfm {

struct LaunchArgs {
  const double* theta;  // P×B device
  int P, B, space;
  const double* panel;  // prepared panel (T × ldp)
  int T, N, np;
  const double* mats;   // N device
  const int* T_use;     // B device or nullptr
  double* out;          // B device
  unsigned int* flags;  // 2 device counters
  double* rec_beta;     // optional trajectories
  double* rec_P;
  hipStream_t stream;
};

// padded maturity count NP the fixed-loading kernel is instantiated for (-1: none)
int fixedz_np_for(int N);
hipError_t launch_fixedz(int kind, const LaunchArgs& a);
hipError_t launch_prep_panel(const double* Y, int N, int T, int np, int ldp, double* out, hipStream_t s);

}  // namespace yfm

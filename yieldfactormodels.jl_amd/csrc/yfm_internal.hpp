// yfm_internal.hpp — launch interface between the C ABI (yfm_capi.hip) and the kernels.
#pragma once
#include "yfm_flags.hpp"
#include <hip/hip_runtime.h>

#include "../../include/yfm.h"

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
  unsigned int* flags;  // this launch's kFlagsPerBank counters (kFlagsPerBank above)
  unsigned int* flags_next = nullptr;  // the other counter bank: zeroed by this launch's first kernel
  double* rec_beta;     // optional trajectories
  double* rec_P;
  double* scratch;      // per-candidate work records (tvl_scratch_bytes, fixedz_scratch_bytes)
  int horizon = 0;      // 0: loglik mode; ≥ 1: trajectory mode (predict / forecast / loss array)
  int rec_len = 0;      // recorded steps per candidate (the last rec_len), stride of rec_beta / rec_P
  int* defer_list = nullptr;   // fixed-loading FP64 kernels → double-double kernel hand-off (B ints)
  int* defer_count = nullptr;  // 1 int, zeroed before the FP64 kernel
  hipStream_t stream;
};

// padded maturity count NP the fixed-loading kernel is instantiated for (-1: none)
int fixedz_np_for(int N);
hipError_t launch_fixedz(int kind, const LaunchArgs& a);
// DNS with N ≤ 32: each filter split over a covariance wave and a mean wave (yfm_split.hip)
bool dns_split_supported(int np);
hipError_t launch_dns_split(const LaunchArgs& a);
// per-candidate initial-state records of the per-lane kernel (GNS5: fixedz_init_kernel), bytes
size_t fixedz_scratch_bytes(int kind, int B);
// fixed-loading models with N beyond the per-lane kernel (yfm_group.hip): filter per lane group
int group_max_n(int kind);
int group_lanes_for(int kind, int N);
hipError_t launch_fixedz_group(int kind, const LaunchArgs& a);
// the deferred fixed-loading candidates (ill-conditioned Z'Z) in double-double arithmetic
// (yfm_fixedz_dd.hip): per-candidate dd records of fixedz_dd_scratch_bytes(kind, B) bytes
size_t fixedz_dd_scratch_bytes(int kind, int B);
hipError_t launch_fixedz_dd(int kind, const LaunchArgs& a, double* rec);
// TVλ EKF kernel (yfm_tvl.hip): lanes per filter for a batch, largest N, launcher.  `share`: launches of this
// size the caller runs concurrently on the device (the estimation driver's chain groups; 1 otherwise)
int tvl_lanes_for(int B, int N, int share = 1);
int tvl_max_n();
size_t tvl_scratch_bytes(int B);
// Maturity jump table for the TVλ exp recurrence (built on the host per lane count L):
// the distinct values d_k of m_{i+L} − m_i and, per maturity i, the index k of its jump.
// K = 0 disables the recurrence (one exp per maturity).
// Power mode (the certified kernel, when the jumps are too many or inexact): every maturity is an exact integer
// multiple k_i·Δ of one step Δ (integer-month grids), so e^{−λm_i} = b^{k_i} with b = e^{−λΔ} — one dd exp per
// step and integer powers of b for the lane starts and the Kp ≤ kTvlPowGaps distinct jump exponents e_q.
constexpr int kTvlGaps = 8;
constexpr int kTvlPowGaps = 16;
struct TvlGaps {
  int K = 0;
  bool exact = false;         // every jump is the exact difference of its two maturities
  const double* d = nullptr;  // device, kTvlGaps
  const int* idx = nullptr;   // device, N
  int Kp = 0;                 // power mode: distinct jump exponents (0: not available)
  double step = 0.0;          // Δ
  const double* e = nullptr;  // device, kTvlPowGaps: the exponents e_q (integers, as doubles)
  const int* pidx = nullptr;  // device, N: each maturity's jump index q
};
hipError_t launch_tvl(const LaunchArgs& a, const TvlGaps& g, int lanes);
// per-candidate FP64 record of the TVλ init kernel (decoded θ + initial state), doubles
constexpr int kRecSigma = 0, kRecDelta = 1, kRecPhi = 5, kRecQ = 21, kRecBeta = 31, kRecP = 35, kRecOk = 45;
constexpr int kRecLen = 48;  // padded to 16-byte multiples
// the same filter in double-double arithmetic (yfm_tvl_dd.hip), YFM_PREC_CERTIFIED: the init
// kernel writes the per-candidate dd records into `rec_dd` (tvl_dd_scratch_bytes(B)); the panel's dd column
// statistics (tvl_dd_colsum_bytes(T)) are made once per panel (yfm_set_panel) or, for a panel of its own
// (get_loss_array's tiled one), by the launch into its scratch (colsum_out).
// tvl_dd_lanes_for picks the lanes per filter (`want` > 0: a requested width, clamped; `share` as tvl_lanes_for)
size_t tvl_dd_scratch_bytes(int B);
size_t tvl_dd_colsum_bytes(int T);
int tvl_dd_lanes_for(int B, int N, int want, int share = 1);
hipError_t launch_tvl_dd_colsum(const double* Y, int N, int T, double* colsum, hipStream_t s);
hipError_t launch_tvl_dd_init(const LaunchArgs& a, double* rec_dd);
hipError_t launch_tvl_dd(const LaunchArgs& a, const double* rec_dd, const double* colsum, const TvlGaps& g, int lanes);
// Trajectory outputs (yfm_predict.hip) from a recorded state trajectory.
struct PredictArgs {
  int kind, M, L, N, P, B, T;
  int ncol;                  // predict: output columns per candidate (T + horizon − 1)
  int horizon;
  const double* theta;       // P×B device
  const double* mats;        // N device
  const int* T_use;          // B device or nullptr
  const double* rec;         // M × rec_len × B trajectory (yfm_kernels.hip / yfm_tvl.hip)
  int rec_len;
  const unsigned char* init_bad;  // B: initialize_filter threw
  double* preds;             // predict: N×ncol×B; forecast: (M+L+N)×h×B; loss array: (T−1)×B
  double* factors;           // predict: M×ncol×B
  double* states;            // predict: L×ncol×B
  double* load1;             // predict: N×ncol×B or nullptr
  double* load2;
  hipStream_t stream;
};
hipError_t launch_init_bad(const double* ll, int B, unsigned char* bad, hipStream_t s);
hipError_t launch_predict_emit(const PredictArgs& a);
hipError_t launch_forecast_emit(const PredictArgs& a);
hipError_t launch_loss_array(const PredictArgs& a, const double* Y, int T1, int passes, unsigned int* flags);
// Extra per-launch work buffers (flags, deferral list, init records) so launches can be in flight
// on several streams of one context at once (yfm_capi.hip; used by the estimation driver).
struct Workspace;
Workspace* workspace_create();
void workspace_destroy(Workspace* w);
int loglik_device_ws(yfm_ctx* ctx, Workspace* ws, int kind, int space, const double* d_theta, int P, int B,
                     const int* d_T_use, double* d_out, hipStream_t s);
// concurrent launches of similar size the caller keeps in flight (the TVλ lane choice sizes the device's share of
// each launch by it); the estimation driver sets its chain-group count and restores 1
void set_lane_share(yfm_ctx* ctx, int share);
// record `msg` as yfm_last_error() for this thread and return `code` (host helpers above the C ABI)
int api_error(int code, const char* msg);
// columns of the context's panel (0 before yfm_set_panel)
int panel_T(const yfm_ctx* ctx);
// a synchronous entry point about to use the context after an asynchronous launch on a caller's stream:
// wait for the device (the caller's stream may be gone, so it is never waited on by handle)
hipError_t settle_foreign_launch(yfm_ctx* ctx);
hipError_t launch_prep_panel(const double* Y, int N, int T, int np, int ldp, double* out, hipStream_t s);

}  // namespace yfm

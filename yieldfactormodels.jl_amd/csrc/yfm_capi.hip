// yfm_capi.hip — the C ABI of libyfm_hip.so (declared in include/yfm.h).
//
// Owns device memory per context (the panel, staging buffers for the host-pointer
// entry points, the flag counters) and launches the kernels of yfm_kernels.hip.
// No torch types, no CPU compute fallback: every result comes from a HIP kernel,
// and a missing/failed device is reported as an error.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/yfm.h"
#include "yfm_internal.hpp"

namespace {

thread_local std::string g_last_error;

int set_error(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define YFM_HIP_CHECK(expr)                                                                      \
  do {                                                                                           \
    hipError_t _e = (expr);                                                                      \
    if (_e != hipSuccess) return set_error(YFM_EHIP, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

int state_dim(int kind) { return kind == YFM_MODEL_DNS ? 3 : kind == YFM_MODEL_TVL ? 4 : kind == YFM_MODEL_GNS5 ? 5 : -1; }
int n_lead(int kind) { return kind == YFM_MODEL_DNS ? 1 : kind == YFM_MODEL_TVL ? 0 : 2; }
// L = length of base.gamma (kalmanbasemodel.jl:58): DNS 1 (dns.jl:18), TVλ 1 (tvλdns.jl:19, never set), GNS5 2
int gamma_dim(int kind) { return kind == YFM_MODEL_GNS5 ? 2 : (state_dim(kind) < 0 ? -1 : 1); }
int param_count(int kind) {
  const int M = state_dim(kind);
  if (M < 0) return -1;
  return n_lead(kind) + 1 + M * (M + 1) / 2 + M + M * M;
}

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipSuccess) cap = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

}  // namespace

// Per-launch device work buffers.  A context owns one; the estimation driver adds one per extra
// concurrent stream (launches in flight on different streams must not share them).
struct yfm::Workspace {
  DevBuf flags;       // 2 banks × kFlagsPerBank unsigned int: n_init_throw, n_neg_inf, deferral list length, n_deferred, steady wave-steps
  int bank = 0;       // the bank of the last launch (the other one is zeroed by that launch's first kernel)
  bool bank_dirty = false;        // the last launch failed: its zeroing of the other bank may not have been enqueued
  hipStream_t last_stream = nullptr;  // the stream of the last launch (compared, never used: it may be gone)
  DevBuf scratch;     // per-candidate work records (TVλ / GNS5 / two-wave DNS init)
  DevBuf scratch_dd;  // TVλ double-double records (YFM_PREC_CERTIFIED)
  DevBuf defer;       // candidates handed from the FP64 fixed-loading kernels to the dd kernel
  DevBuf scratch_fd;  // their double-double records (yfm_fixedz_dd.hip)
};

struct yfm_ctx {
  int device = 0;
  int precision = YFM_PREC_CERTIFIED;  // TVλ arithmetic (yfm_set_precision)
  int lane_share = 1;                  // concurrent launches in flight (yfm::set_lane_share)
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;  // θ uploads of pipelined host-pointer batches (created lazily)
  // panel
  int N = 0, T = 0, np = 0, ldp = 0;
  DevBuf panel, mats, raw;
  DevBuf colsum;  // the panel's dd column statistics (certified TVλ), made by yfm_set_panel
  // staging for host-pointer calls
  DevBuf theta, out, tuse, rec_beta, rec_P;
  DevBuf flags;  // 2 banks × kFlagsPerBank unsigned int: n_init_throw, n_neg_inf, deferral list length, n_deferred, steady wave-steps
  int bank = 0;  // the bank of the last launch (the other one is zeroed by that launch's first kernel)
  bool bank_dirty = false;            // as Workspace::bank_dirty
  hipStream_t last_stream = nullptr;  // as Workspace::last_stream
  DevBuf scratch;  // per-candidate work records (TVλ init)
  DevBuf scratch_dd;  // TVλ double-double records (YFM_PREC_CERTIFIED)
  DevBuf traj, init_bad;       // trajectory-mode state records, per-candidate init-throw marks
  DevBuf defer;                // candidates handed from the FP64 fixed-loading kernels to the dd kernel
  DevBuf scratch_fd;           // their double-double records (yfm_fixedz_dd.hip)
  DevBuf tiled_raw, tiled_panel;  // get_loss_array with K > 1 passes: the panel tiled K times
  // TVλ maturity-jump tables, one per lane count L = 2^l (built lazily, reset by set_panel)
  std::vector<double> mats_host;
  int gap_K[7] = {-1, -1, -1, -1, -1, -1, -1};
  bool gap_exact[7] = {};
  DevBuf gap_buf[7];
  int pow_K[7] = {};       // power-mode tables (TvlGaps::Kp), built with the jump tables
  double pow_step = 0.0;   // Δ (0: the maturities are not integer multiples of one step)
  DevBuf pow_buf[7];
};

namespace {

// host-pointer pipelining (yfm_loglik_batch): chunk ≥ 2 per-lane waves per SIMD, ≤ 8 chunks
constexpr int kPipeChunk = 131072;
constexpr int kPipeMaxChunks = 8;

int check_ctx(yfm_ctx* ctx) {
  if (!ctx) return set_error(YFM_EINVAL, "null context");
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return set_error(YFM_EHIP, "hipSetDevice(%d): %s", ctx->device, hipGetErrorString(e));
  return YFM_OK;
}

int check_batch(yfm_ctx* ctx, int kind, int space, int P, int B) {
  if (state_dim(kind) < 0) return set_error(YFM_EINVAL, "unknown model_kind %d", kind);
  if (space != YFM_THETA_UNCONSTRAINED && space != YFM_THETA_CONSTRAINED)
    return set_error(YFM_EINVAL, "unknown param_space %d", space);
  if (P != param_count(kind))
    return set_error(YFM_EINVAL, "P = %d but model_kind %d has %d parameters", P, kind, param_count(kind));
  if (B < 0) return set_error(YFM_EINVAL, "B = %d < 0", B);
  if (ctx->T <= 0) return set_error(YFM_ENOPANEL, "no panel: call yfm_set_panel first");
  if (kind == YFM_MODEL_TVL) {
    if (ctx->N > yfm::tvl_max_n())
      return set_error(YFM_EUNSUPPORTED, "N = %d maturities exceeds the TVλ kernel's %d", ctx->N, yfm::tvl_max_n());
    return YFM_OK;
  }
  if (yfm::fixedz_np_for(ctx->N) < 0 && ctx->N > yfm::group_max_n(kind))
    return set_error(YFM_EUNSUPPORTED, "N = %d maturities exceeds the fixed-loading kernels' %d", ctx->N,
                     yfm::group_max_n(kind));
  return YFM_OK;
}

// Jump table of the TVλ exp recurrence for lane count L: distinct m_{i+L} − m_i (exact
// equality) and each maturity's index; K = 0 when there are more than yfm::kTvlGaps.
int tvl_gaps(yfm_ctx* ctx, int L, yfm::TvlGaps& g) {
  int l = 0;
  while ((1 << l) < L) ++l;
  if (ctx->gap_K[l] < 0) {
    const int N = ctx->N;
    std::vector<double> d;
    std::vector<int> idx(N, 0);
    bool ok = true;
    bool exact = true;
    for (int i = 0; i + L < N && ok; ++i) {
      const double hi = ctx->mats_host[i + L], lo = ctx->mats_host[i];
      const double gap = hi - lo;
      // TwoSum error of the subtraction: the double-double filter needs the jumps exactly
      const double bb = gap - hi;
      exact = exact && ((hi - (gap - bb)) + (-lo - bb)) == 0.0;
      int k = 0;
      while (k < (int)d.size() && d[k] != gap) ++k;
      if (k == (int)d.size()) {
        if ((int)d.size() == yfm::kTvlGaps) ok = false;
        else d.push_back(gap);
      }
      idx[i] = k;
    }
    int K = ok ? (int)d.size() : 0;
    if (K == 0 && ok) K = 1, d.push_back(0.0);  // N ≤ L: every lane has at most one maturity
    d.resize(yfm::kTvlGaps, 0.0);
    if (K > 0) {
      YFM_HIP_CHECK(ctx->gap_buf[l].ensure(sizeof(double) * yfm::kTvlGaps + sizeof(int) * N));
      char* base = static_cast<char*>(ctx->gap_buf[l].p);
      YFM_HIP_CHECK(hipMemcpy(base, d.data(), sizeof(double) * yfm::kTvlGaps, hipMemcpyHostToDevice));
      YFM_HIP_CHECK(hipMemcpy(base + sizeof(double) * yfm::kTvlGaps, idx.data(), sizeof(int) * N,
                              hipMemcpyHostToDevice));
    }
    ctx->gap_K[l] = K;
    ctx->gap_exact[l] = exact;
    // power mode: every maturity an integer multiple of Δ = gcd (exactly, as doubles: integer-valued and < 2^31)
    ctx->pow_K[l] = 0;
    long long gcd = 0;
    bool integral = N > 0;
    for (int i = 0; i < N && integral; ++i) {
      const double m = ctx->mats_host[i];
      integral = m > 0.0 && m < 2147483648.0 && m == std::floor(m);
      long long a = integral ? (long long)m : 0, b = gcd;
      while (b) {
        const long long t = a % b;
        a = b;
        b = t;
      }
      gcd = a;
    }
    ctx->pow_step = integral ? (double)gcd : 0.0;
    if (integral && N > L) {
      std::vector<double> e;
      std::vector<int> pidx(N, 0);
      bool fits = true;
      for (int i = 0; i + L < N && fits; ++i) {
        const double q = (ctx->mats_host[i + L] - ctx->mats_host[i]) / (double)gcd;  // exact: integers < 2^31
        int k = 0;
        while (k < (int)e.size() && e[k] != q) ++k;
        if (k == (int)e.size()) {
          if ((int)e.size() == yfm::kTvlPowGaps || !(q >= 1.0 && q < 512.0)) fits = false;
          else e.push_back(q);
        }
        pidx[i] = k;
      }
      if (fits) {
        e.resize(yfm::kTvlPowGaps, 0.0);
        YFM_HIP_CHECK(ctx->pow_buf[l].ensure(sizeof(double) * yfm::kTvlPowGaps + sizeof(int) * N));
        char* base = static_cast<char*>(ctx->pow_buf[l].p);
        YFM_HIP_CHECK(hipMemcpy(base, e.data(), sizeof(double) * yfm::kTvlPowGaps, hipMemcpyHostToDevice));
        YFM_HIP_CHECK(hipMemcpy(base + sizeof(double) * yfm::kTvlPowGaps, pidx.data(), sizeof(int) * N,
                                hipMemcpyHostToDevice));
        int Kp = 0;
        while (Kp < yfm::kTvlPowGaps && e[Kp] != 0.0) ++Kp;
        ctx->pow_K[l] = Kp;
      }
    }
  }
  g.K = ctx->gap_K[l];
  g.exact = ctx->gap_exact[l];
  if (g.K > 0) {
    char* base = static_cast<char*>(ctx->gap_buf[l].p);
    g.d = reinterpret_cast<const double*>(base);
    g.idx = reinterpret_cast<const int*>(base + sizeof(double) * yfm::kTvlGaps);
  }
  g.Kp = ctx->pow_K[l];
  if (g.Kp > 0) {
    char* base = static_cast<char*>(ctx->pow_buf[l].p);
    g.step = ctx->pow_step;
    g.e = reinterpret_cast<const double*>(base);
    g.pidx = reinterpret_cast<const int*>(base + sizeof(double) * yfm::kTvlPowGaps);
  }
  if (const char* ov = std::getenv("YFM_TVL_EXP")) {  // diagnostic: force one exp per maturity
    if (std::atoi(ov) == 1) g.K = g.Kp = 0;
  }
  return YFM_OK;
}

// A panel other than the context's (get_loss_array's K-times tiled panel).
struct PanelView {
  const double* raw;
  const double* panel;
  int T;
};

int launch_impl(yfm_ctx* ctx, int kind, int space, const double* d_theta, int P, int B, const int* d_T_use,
                double* d_out, double* d_rb, double* d_rP, hipStream_t s, int horizon, int rec_len,
                const PanelView* pv, bool reset_flags, yfm::Workspace* ws);

// Counters [n_init_throw, n_neg_inf, defer_count, n_deferred, steady] in two banks: a launch uses the bank
// its predecessor zeroed (its first kernel zeroes the other one), so no memset is enqueued per call.
// That hand-off only holds when the predecessor's kernels were all enqueued (bank_dirty otherwise) and ran
// on the same stream; after a failed launch or on a stream change this launch zeroes its bank itself, on
// its own stream.  Launches on different streams are ordered by the caller (include/yfm.h: a context's
// scratch serves one launch at a time), so no event is recorded per launch — one was, in an earlier
// round-4 build, and cost 4.7 µs of every config-2 call (profiles/r4/exp1/) — and the library never
// touches the previous launch's stream (the estimator destroys its group streams).  The bank index flips
// only once the launch succeeded.  A pipelined chunk continues its batch's counters and only resets the
// deferral list length.
int launch(yfm_ctx* ctx, int kind, int space, const double* d_theta, int P, int B, const int* d_T_use,
           double* d_out, double* d_rb, double* d_rP, hipStream_t s, int horizon = 0, int rec_len = 0,
           const PanelView* pv = nullptr, bool reset_flags = true, yfm::Workspace* ws = nullptr) {
  DevBuf& w_flags = ws ? ws->flags : ctx->flags;
  int& w_bank = ws ? ws->bank : ctx->bank;
  bool& dirty = ws ? ws->bank_dirty : ctx->bank_dirty;
  hipStream_t& last = ws ? ws->last_stream : ctx->last_stream;
  unsigned int* fb = static_cast<unsigned int*>(w_flags.p);
  // the context's own (synchronous) stream after a launch on a caller's stream: that launch may still run
  if (!ws && s == ctx->stream) YFM_HIP_CHECK(yfm::settle_foreign_launch(ctx));
  if (reset_flags && (dirty || s != last)) {
    YFM_HIP_CHECK(hipMemsetAsync(fb + yfm::kFlagsPerBank * (w_bank ^ 1), 0, yfm::kFlagsPerBank * sizeof(unsigned int), s));
    dirty = false;
  }
  const int r = launch_impl(ctx, kind, space, d_theta, P, B, d_T_use, d_out, d_rb, d_rP, s, horizon, rec_len, pv,
                            reset_flags, ws);
  if (r != YFM_OK) {
    dirty = true;
    return r;
  }
  if (reset_flags) {
    w_bank ^= 1;
    last = s;
  }
  return YFM_OK;
}

int launch_impl(yfm_ctx* ctx, int kind, int space, const double* d_theta, int P, int B, const int* d_T_use,
                double* d_out, double* d_rb, double* d_rP, hipStream_t s, int horizon, int rec_len,
                const PanelView* pv, bool reset_flags, yfm::Workspace* ws) {
  DevBuf& w_flags = ws ? ws->flags : ctx->flags;
  const int w_bank = (ws ? ws->bank : ctx->bank) ^ (reset_flags ? 1 : 0);  // the bank this launch uses
  DevBuf& w_scratch = ws ? ws->scratch : ctx->scratch;
  DevBuf& w_scratch_dd = ws ? ws->scratch_dd : ctx->scratch_dd;
  DevBuf& w_defer = ws ? ws->defer : ctx->defer;
  DevBuf& w_scratch_fd = ws ? ws->scratch_fd : ctx->scratch_fd;
  unsigned int* fb = static_cast<unsigned int*>(w_flags.p);
  unsigned int* flags_next = nullptr;
  if (reset_flags) {
    flags_next = fb + yfm::kFlagsPerBank * (w_bank ^ 1);
  } else {
    YFM_HIP_CHECK(hipMemsetAsync(fb + yfm::kFlagsPerBank * w_bank + 2, 0, sizeof(unsigned int), s));
  }
  if (B == 0) {  // no kernel runs: zero both banks here
    YFM_HIP_CHECK(hipMemsetAsync(fb, 0, 2 * yfm::kFlagsPerBank * sizeof(unsigned int), s));
    return YFM_OK;
  }
  yfm::LaunchArgs a;
  a.theta = d_theta;
  a.P = P;
  a.B = B;
  a.space = space;
  a.panel = static_cast<const double*>(ctx->panel.p);
  a.raw = static_cast<const double*>(ctx->raw.p);
  a.T = ctx->T;
  a.N = ctx->N;
  a.np = ctx->np;
  a.ldp = ctx->ldp;
  a.mats = static_cast<const double*>(ctx->mats.p);
  a.T_use = d_T_use;
  a.out = d_out;
  a.flags = fb + yfm::kFlagsPerBank * w_bank;
  a.flags_next = flags_next;
  a.rec_beta = d_rb;
  a.rec_P = d_rP;
  a.scratch = nullptr;
  a.horizon = horizon;
  a.rec_len = d_rb ? (rec_len > 0 ? rec_len : ctx->T - 1) : 0;
  if (pv) {
    a.raw = pv->raw;
    a.panel = pv->panel;
    a.T = pv->T;
  }
  a.stream = s;
  hipError_t e;
  if (kind == YFM_MODEL_TVL) {
    int lanes = yfm::tvl_lanes_for(B, ctx->N, ctx->lane_share);
    if (const char* ov = std::getenv("YFM_TVL_LANES")) {  // tuning override: 1, 2, 4, …, 64
      const int l = std::atoi(ov);
      if (l >= 1 && l <= 64 && (l & (l - 1)) == 0) lanes = l;
    }
    yfm::TvlGaps g;
    if (ctx->precision == YFM_PREC_CERTIFIED) {
      lanes = yfm::tvl_dd_lanes_for(B, ctx->N, std::getenv("YFM_TVL_LANES") ? lanes : 0, ctx->lane_share);
      // the context's panel has its column statistics already; a panel of the launch's own gets them here
      const bool own_panel = pv && pv->raw != static_cast<const double*>(ctx->raw.p);
      const size_t rec_bytes = yfm::tvl_dd_scratch_bytes(B);
      YFM_HIP_CHECK(w_scratch_dd.ensure(rec_bytes + (own_panel ? yfm::tvl_dd_colsum_bytes(a.T) : 0)));
      double* rdd = static_cast<double*>(w_scratch_dd.p);
      const double* colsum = static_cast<const double*>(ctx->colsum.p);
      if (own_panel) {
        double* cs = rdd + rec_bytes / sizeof(double);
        YFM_HIP_CHECK(yfm::launch_tvl_dd_colsum(a.raw, a.N, a.T, cs, s));
        colsum = cs;
      }
      if (int r = tvl_gaps(ctx, lanes, g)) return r;
      e = yfm::launch_tvl_dd_init(a, rdd);
      if (e == hipSuccess) e = yfm::launch_tvl_dd(a, rdd, colsum, g, lanes);
    } else {
      YFM_HIP_CHECK(w_scratch.ensure(yfm::tvl_scratch_bytes(B)));
      a.scratch = static_cast<double*>(w_scratch.p);
      if (int r = tvl_gaps(ctx, lanes, g)) return r;
      e = yfm::launch_tvl(a, g, lanes);
    }
  } else {
    // N ≤ 64: one filter per lane (MFMA Z'y); larger N: one filter per lane group.  Either defers
    // the candidates with an ill-conditioned Z'Z, which the double-double kernel then evaluates
    YFM_HIP_CHECK(w_defer.ensure(sizeof(int) * (size_t)B));
    YFM_HIP_CHECK(w_scratch_fd.ensure(yfm::fixedz_dd_scratch_bytes(kind, B)));
    a.defer_count = reinterpret_cast<int*>(a.flags + 2);  // zero (a fresh bank, or reset above)
    a.defer_list = static_cast<int*>(w_defer.p);
    if (yfm::fixedz_np_for(ctx->N) > 0) {
      if (const size_t sb = yfm::fixedz_scratch_bytes(kind, B)) {
        YFM_HIP_CHECK(w_scratch.ensure(sb));
        a.scratch = static_cast<double*>(w_scratch.p);
      }
      e = yfm::launch_fixedz(kind, a);
    } else {
      e = yfm::launch_fixedz_group(kind, a);
    }
    if (e == hipSuccess) e = yfm::launch_fixedz_dd(kind, a, static_cast<double*>(w_scratch_fd.p));
  }
  if (e != hipSuccess) return set_error(YFM_EHIP, "kernel launch: %s", hipGetErrorString(e));
  return YFM_OK;
}

// Upload θ (and T_use) for a host-pointer call; returns the device pointers.
int stage_inputs(yfm_ctx* ctx, const double* theta, int P, int B, const int* T_use, const double** d_th,
                 const int** d_tu) {
  const size_t nb = (size_t)(B > 0 ? B : 1);
  YFM_HIP_CHECK(ctx->theta.ensure(sizeof(double) * (size_t)P * nb));
  YFM_HIP_CHECK(ctx->out.ensure(sizeof(double) * nb));
  if (B > 0)
    YFM_HIP_CHECK(hipMemcpyAsync(ctx->theta.p, theta, sizeof(double) * (size_t)P * B, hipMemcpyHostToDevice,
                                 ctx->stream));
  *d_th = static_cast<const double*>(ctx->theta.p);
  *d_tu = nullptr;
  if (T_use && B > 0) {
    YFM_HIP_CHECK(ctx->tuse.ensure(sizeof(int) * nb));
    YFM_HIP_CHECK(hipMemcpyAsync(ctx->tuse.p, T_use, sizeof(int) * B, hipMemcpyHostToDevice, ctx->stream));
    *d_tu = static_cast<const int*>(ctx->tuse.p);
  }
  return YFM_OK;
}

// Trajectory mode: run the filter kernel recording the last rec_len states of every
// candidate into ctx->traj and mark the candidates whose initialize_filter threw.
int run_trajectory(yfm_ctx* ctx, int kind, int space, const double* d_th, int P, int B, const int* d_tu,
                   int horizon, int rec_len, const PanelView* pv = nullptr) {
  const int M = state_dim(kind);
  const size_t n = (size_t)B * rec_len * M;
  YFM_HIP_CHECK(ctx->traj.ensure(sizeof(double) * (n > 0 ? n : 1)));
  YFM_HIP_CHECK(ctx->init_bad.ensure((size_t)(B > 0 ? B : 1)));
  YFM_HIP_CHECK(hipMemsetAsync(ctx->traj.p, 0xff, sizeof(double) * n, ctx->stream));  // NaN fill
  if (int r = launch(ctx, kind, space, d_th, P, B, d_tu, static_cast<double*>(ctx->out.p),
                     static_cast<double*>(ctx->traj.p), nullptr, ctx->stream, horizon, rec_len, pv))
    return r;
  YFM_HIP_CHECK(yfm::launch_init_bad(static_cast<const double*>(ctx->out.p), B,
                                     static_cast<unsigned char*>(ctx->init_bad.p), ctx->stream));
  return YFM_OK;
}

yfm::PredictArgs predict_args(yfm_ctx* ctx, int kind, const double* d_th, int P, int B, const int* d_tu,
                              int horizon, int rec_len) {
  yfm::PredictArgs a{};
  a.kind = kind;
  a.M = state_dim(kind);
  a.L = gamma_dim(kind);
  a.N = ctx->N;
  a.P = P;
  a.B = B;
  a.T = ctx->T;
  a.horizon = horizon;
  a.ncol = ctx->T + horizon - 1;
  a.theta = d_th;
  a.mats = static_cast<const double*>(ctx->mats.p);
  a.T_use = d_tu;
  a.rec = static_cast<const double*>(ctx->traj.p);
  a.rec_len = rec_len;
  a.init_bad = static_cast<const unsigned char*>(ctx->init_bad.p);
  a.stream = ctx->stream;
  return a;
}

int validate_tuse(const int* T_use, int B, int T) {
  if (!T_use) return YFM_OK;
  for (int b = 0; b < B; ++b)
    if (T_use[b] < 1 || T_use[b] > T)
      return set_error(YFM_EINVAL, "T_use[%d] = %d outside [1, %d]", b, T_use[b], T);
  return YFM_OK;
}

}  // namespace

namespace yfm {
int api_error(int code, const char* msg) { return set_error(code, "%s", msg); }
int panel_T(const yfm_ctx* ctx) { return ctx ? ctx->T : 0; }

hipError_t settle_foreign_launch(yfm_ctx* ctx) {
  if (!ctx || !ctx->last_stream || ctx->last_stream == ctx->stream) return hipSuccess;
  const hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) ctx->last_stream = nullptr;  // nothing of the context is in flight any more
  return e;
}
}  // namespace yfm

extern "C" {

int yfm_abi_version(void) { return YFM_ABI_VERSION; }
int yfm_param_count(int model_kind) { return param_count(model_kind); }
int yfm_state_dim(int model_kind) { return state_dim(model_kind); }
const char* yfm_last_error(void) { return g_last_error.c_str(); }

yfm_ctx* yfm_create(int hip_device) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) {
    set_error(YFM_EHIP, "no HIP device available (%s)", hipGetErrorString(e));
    return nullptr;
  }
  if (hip_device < 0 || hip_device >= n) {
    set_error(YFM_EINVAL, "hip_device %d out of range [0, %d)", hip_device, n);
    return nullptr;
  }
  if (hipSetDevice(hip_device) != hipSuccess) {
    set_error(YFM_EHIP, "hipSetDevice(%d) failed", hip_device);
    return nullptr;
  }
  yfm_ctx* ctx = new yfm_ctx();
  ctx->device = hip_device;
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      ctx->flags.ensure(2 * yfm::kFlagsPerBank * sizeof(unsigned int)) != hipSuccess) {
    set_error(YFM_EHIP, "context allocation failed on device %d", hip_device);
    yfm_destroy(ctx);
    return nullptr;
  }
  (void)hipMemset(ctx->flags.p, 0, 2 * yfm::kFlagsPerBank * sizeof(unsigned int));
  return ctx;
}

void yfm_destroy(yfm_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (DevBuf* b : {&ctx->panel, &ctx->mats, &ctx->raw, &ctx->theta, &ctx->out, &ctx->tuse, &ctx->rec_beta,
                    &ctx->rec_P, &ctx->flags, &ctx->scratch})
    b->release();
  for (DevBuf* b : {&ctx->traj, &ctx->init_bad, &ctx->tiled_raw, &ctx->tiled_panel, &ctx->defer, &ctx->scratch_fd})
    b->release();
  ctx->scratch_dd.release();
  for (DevBuf& b : ctx->gap_buf) b.release();
  for (DevBuf& b : ctx->pow_buf) b.release();
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->copy_stream) (void)hipStreamDestroy(ctx->copy_stream);
  delete ctx;
}

void* yfm_alloc_host(size_t bytes) {
  void* p = nullptr;
  hipError_t e = hipHostMalloc(&p, bytes > 0 ? bytes : 1, hipHostMallocPortable);
  if (e != hipSuccess) {
    set_error(YFM_EHIP, "hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
    return nullptr;
  }
  return p;
}

int yfm_free_host(void* p) {
  if (!p) return YFM_OK;
  YFM_HIP_CHECK(hipHostFree(p));
  return YFM_OK;
}

int yfm_set_precision(yfm_ctx* ctx, int precision) {
  if (int r = check_ctx(ctx)) return r;
  if (precision != YFM_PREC_CERTIFIED && precision != YFM_PREC_FP64)
    return set_error(YFM_EINVAL, "unknown precision %d", precision);
  ctx->precision = precision;
  return YFM_OK;
}

int yfm_get_precision(yfm_ctx* ctx) {
  if (!ctx) return set_error(YFM_EINVAL, "null context");
  return ctx->precision;
}

int yfm_set_panel(yfm_ctx* ctx, const double* Y, int N, int T, const double* maturities) {
  if (int r = check_ctx(ctx)) return r;
  YFM_HIP_CHECK(yfm::settle_foreign_launch(ctx));  // a launch on a caller's stream may still read the panel
  if (!Y || !maturities) return set_error(YFM_EINVAL, "null Y or maturities");
  if (N < 1 || T < 1) return set_error(YFM_EINVAL, "N = %d, T = %d must be >= 1", N, T);
  const int np = yfm::fixedz_np_for(N);
  const int npad = np > 0 ? np : ((N + 7) / 8) * 8;
  const int ldp = npad + 4;
  YFM_HIP_CHECK(ctx->raw.ensure(sizeof(double) * (size_t)N * T));
  YFM_HIP_CHECK(ctx->panel.ensure(sizeof(double) * (size_t)ldp * T));
  YFM_HIP_CHECK(ctx->mats.ensure(sizeof(double) * (size_t)N));
  YFM_HIP_CHECK(hipMemcpyAsync(ctx->raw.p, Y, sizeof(double) * (size_t)N * T, hipMemcpyHostToDevice, ctx->stream));
  YFM_HIP_CHECK(hipMemcpyAsync(ctx->mats.p, maturities, sizeof(double) * N, hipMemcpyHostToDevice, ctx->stream));
  YFM_HIP_CHECK(yfm::launch_prep_panel(static_cast<const double*>(ctx->raw.p), N, T, npad, ldp,
                                       static_cast<double*>(ctx->panel.p), ctx->stream));
  YFM_HIP_CHECK(ctx->colsum.ensure(yfm::tvl_dd_colsum_bytes(T)));
  YFM_HIP_CHECK(yfm::launch_tvl_dd_colsum(static_cast<const double*>(ctx->raw.p), N, T,
                                          static_cast<double*>(ctx->colsum.p), ctx->stream));
  YFM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  ctx->N = N;
  ctx->T = T;
  ctx->mats_host.assign(maturities, maturities + N);
  for (int& k : ctx->gap_K) k = -1;
  ctx->np = npad;
  ctx->ldp = ldp;
  return YFM_OK;
}

int yfm_loglik_batch(yfm_ctx* ctx, int model_kind, int param_space, const double* theta, int P, int B,
                     const int* T_use, double* loglik_out) {
  if (int r = check_ctx(ctx)) return r;
  if (int r = check_batch(ctx, model_kind, param_space, P, B)) return r;
  if (B > 0 && (!theta || !loglik_out)) return set_error(YFM_EINVAL, "null theta or loglik_out");
  if (int r = validate_tuse(T_use, B, ctx->T)) return r;
  const size_t nb = (size_t)(B > 0 ? B : 1);
  YFM_HIP_CHECK(ctx->theta.ensure(sizeof(double) * (size_t)P * nb));
  YFM_HIP_CHECK(ctx->out.ensure(sizeof(double) * nb));
  if (T_use && B > 0) YFM_HIP_CHECK(ctx->tuse.ensure(sizeof(int) * nb));
  double* d_th = static_cast<double*>(ctx->theta.p);
  double* d_out = static_cast<double*>(ctx->out.p);
  int* d_tu = T_use ? static_cast<int*>(ctx->tuse.p) : nullptr;
  // Batches that fill the chip several times over are pipelined: chunk k+1's θ is uploaded on
  // the copy stream while chunk k's filter runs on the context stream (each chunk still holds
  // ≥ 2 waves per SIMD of candidates).  Evaluations are independent, so the logliks are the
  // same bits as one launch; the flags accumulate over the chunks.
  int chunk = B;
  if (model_kind != YFM_MODEL_TVL && B >= 2 * kPipeChunk) {
    chunk = std::max(kPipeChunk, (B + kPipeMaxChunks - 1) / kPipeMaxChunks);
    if (!ctx->copy_stream) YFM_HIP_CHECK(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
  }
  if (chunk < B) {
    const int nchunks = (B + chunk - 1) / chunk;
    std::vector<hipEvent_t> ev(nchunks, nullptr);
    int rc = YFM_OK;
    for (int k = 0; k < nchunks && rc == YFM_OK; ++k) {
      const int b0 = k * chunk, nbk = std::min(chunk, B - b0);
      hipError_t e = hipEventCreateWithFlags(&ev[k], hipEventDisableTiming);
      if (e == hipSuccess)
        e = hipMemcpyAsync(d_th + (size_t)P * b0, theta + (size_t)P * b0, sizeof(double) * (size_t)P * nbk,
                           hipMemcpyHostToDevice, ctx->copy_stream);
      if (e == hipSuccess && d_tu)
        e = hipMemcpyAsync(d_tu + b0, T_use + b0, sizeof(int) * nbk, hipMemcpyHostToDevice, ctx->copy_stream);
      if (e == hipSuccess) e = hipEventRecord(ev[k], ctx->copy_stream);
      if (e == hipSuccess) e = hipStreamWaitEvent(ctx->stream, ev[k], 0);
      if (e != hipSuccess) {
        rc = set_error(YFM_EHIP, "pipelined upload: %s", hipGetErrorString(e));
        break;
      }
      rc = launch(ctx, model_kind, param_space, d_th + (size_t)P * b0, P, nbk, d_tu ? d_tu + b0 : nullptr,
                  d_out + b0, nullptr, nullptr, ctx->stream, 0, 0, nullptr, k == 0);
    }
    if (rc == YFM_OK) {
      hipError_t e = hipMemcpyAsync(loglik_out, d_out, sizeof(double) * B, hipMemcpyDeviceToHost, ctx->stream);
      if (e != hipSuccess) rc = set_error(YFM_EHIP, "hipMemcpyAsync: %s", hipGetErrorString(e));
    }
    (void)hipStreamSynchronize(ctx->copy_stream);
    hipError_t e = hipStreamSynchronize(ctx->stream);
    for (hipEvent_t x : ev)
      if (x) (void)hipEventDestroy(x);
    if (rc == YFM_OK && e != hipSuccess) rc = set_error(YFM_EHIP, "hipStreamSynchronize: %s", hipGetErrorString(e));
    return rc;
  }
  if (B > 0)
    YFM_HIP_CHECK(hipMemcpyAsync(d_th, theta, sizeof(double) * (size_t)P * B, hipMemcpyHostToDevice, ctx->stream));
  if (d_tu && B > 0)
    YFM_HIP_CHECK(hipMemcpyAsync(d_tu, T_use, sizeof(int) * B, hipMemcpyHostToDevice, ctx->stream));
  if (int r = launch(ctx, model_kind, param_space, d_th, P, B, d_tu, d_out, nullptr, nullptr, ctx->stream))
    return r;
  if (B > 0)
    YFM_HIP_CHECK(hipMemcpyAsync(loglik_out, d_out, sizeof(double) * B, hipMemcpyDeviceToHost, ctx->stream));
  YFM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  return YFM_OK;
}


int yfm_loglik_batch_device(yfm_ctx* ctx, int model_kind, int param_space, const double* d_theta, int P, int B,
                            const int* d_T_use, double* d_loglik_out, void* hip_stream) {
  if (int r = check_ctx(ctx)) return r;
  if (int r = check_batch(ctx, model_kind, param_space, P, B)) return r;
  if (B > 0 && (!d_theta || !d_loglik_out)) return set_error(YFM_EINVAL, "null d_theta or d_loglik_out");
  return launch(ctx, model_kind, param_space, d_theta, P, B, d_T_use, d_loglik_out, nullptr, nullptr,
                static_cast<hipStream_t>(hip_stream));
}

int yfm_filter_states(yfm_ctx* ctx, int model_kind, int param_space, const double* theta, int P, int B,
                      const int* T_use, double* beta_out, double* P_out, double* loglik_out) {
  if (int r = check_ctx(ctx)) return r;
  if (int r = check_batch(ctx, model_kind, param_space, P, B)) return r;
  if (B > 0 && (!theta || !beta_out || !P_out || !loglik_out)) return set_error(YFM_EINVAL, "null pointer argument");
  if (int r = validate_tuse(T_use, B, ctx->T)) return r;
  if (B == 0 || ctx->T < 2) {
    return yfm_loglik_batch(ctx, model_kind, param_space, theta, P, B, T_use, loglik_out);
  }
  const int M = state_dim(model_kind);
  const size_t steps = (size_t)(ctx->T - 1) * B;
  YFM_HIP_CHECK(ctx->theta.ensure(sizeof(double) * (size_t)P * B));
  YFM_HIP_CHECK(ctx->out.ensure(sizeof(double) * B));
  YFM_HIP_CHECK(ctx->rec_beta.ensure(sizeof(double) * steps * M));
  YFM_HIP_CHECK(ctx->rec_P.ensure(sizeof(double) * steps * M * M));
  YFM_HIP_CHECK(hipMemsetAsync(ctx->rec_beta.p, 0xff, sizeof(double) * steps * M, ctx->stream));  // NaN fill
  YFM_HIP_CHECK(hipMemsetAsync(ctx->rec_P.p, 0xff, sizeof(double) * steps * M * M, ctx->stream));
  YFM_HIP_CHECK(hipMemcpyAsync(ctx->theta.p, theta, sizeof(double) * (size_t)P * B, hipMemcpyHostToDevice,
                               ctx->stream));
  const int* d_tuse = nullptr;
  if (T_use) {
    YFM_HIP_CHECK(ctx->tuse.ensure(sizeof(int) * B));
    YFM_HIP_CHECK(hipMemcpyAsync(ctx->tuse.p, T_use, sizeof(int) * B, hipMemcpyHostToDevice, ctx->stream));
    d_tuse = static_cast<const int*>(ctx->tuse.p);
  }
  if (int r = launch(ctx, model_kind, param_space, static_cast<const double*>(ctx->theta.p), P, B, d_tuse,
                     static_cast<double*>(ctx->out.p), static_cast<double*>(ctx->rec_beta.p),
                     static_cast<double*>(ctx->rec_P.p), ctx->stream, 0, ctx->T - 1))
    return r;
  YFM_HIP_CHECK(hipMemcpyAsync(loglik_out, ctx->out.p, sizeof(double) * B, hipMemcpyDeviceToHost, ctx->stream));
  YFM_HIP_CHECK(hipMemcpyAsync(beta_out, ctx->rec_beta.p, sizeof(double) * steps * M, hipMemcpyDeviceToHost,
                               ctx->stream));
  YFM_HIP_CHECK(hipMemcpyAsync(P_out, ctx->rec_P.p, sizeof(double) * steps * M * M, hipMemcpyDeviceToHost,
                               ctx->stream));
  YFM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  return YFM_OK;
}

int yfm_last_batch_flags(yfm_ctx* ctx, long long* n_init_throw, long long* n_neg_inf) {
  if (int r = check_ctx(ctx)) return r;
  unsigned int h[2] = {0, 0};
  YFM_HIP_CHECK(hipMemcpy(h, static_cast<unsigned int*>(ctx->flags.p) + yfm::kFlagsPerBank * ctx->bank, sizeof(h), hipMemcpyDeviceToHost));
  if (n_init_throw) *n_init_throw = h[0];
  if (n_neg_inf) *n_neg_inf = h[1];
  return YFM_OK;
}

int yfm_last_batch_deferred(yfm_ctx* ctx, long long* n_deferred) {
  if (int r = check_ctx(ctx)) return r;
  unsigned int h[4] = {0, 0, 0, 0};
  YFM_HIP_CHECK(hipMemcpy(h, static_cast<unsigned int*>(ctx->flags.p) + yfm::kFlagsPerBank * ctx->bank, sizeof(h), hipMemcpyDeviceToHost));
  if (n_deferred) *n_deferred = h[3];
  return YFM_OK;
}

int yfm_last_batch_steady(yfm_ctx* ctx, long long* steady_wave_steps) {
  if (int r = check_ctx(ctx)) return r;
  unsigned int h[5] = {0, 0, 0, 0, 0};
  YFM_HIP_CHECK(hipMemcpy(h, static_cast<unsigned int*>(ctx->flags.p) + yfm::kFlagsPerBank * ctx->bank, sizeof(h),
                          hipMemcpyDeviceToHost));
  if (steady_wave_steps) *steady_wave_steps = h[4];
  return YFM_OK;
}

int yfm_gamma_dim(int model_kind) { return gamma_dim(model_kind); }

int yfm_predict(yfm_ctx* ctx, int model_kind, int param_space, const double* theta, int P, int B, const int* T_use,
                int horizon, double* preds, double* factors, double* states, double* loadings_1,
                double* loadings_2) {
  if (int r = check_ctx(ctx)) return r;
  if (int r = check_batch(ctx, model_kind, param_space, P, B)) return r;
  if (horizon < 1) return set_error(YFM_EINVAL, "horizon = %d < 1", horizon);
  if (B > 0 && (!theta || !preds || !factors || !states)) return set_error(YFM_EINVAL, "null pointer argument");
  if (int r = validate_tuse(T_use, B, ctx->T)) return r;
  if (B == 0) return YFM_OK;
  const int M = state_dim(model_kind), L = gamma_dim(model_kind), N = ctx->N;
  const int rec_len = ctx->T + horizon;  // every step of the longest candidate
  const size_t ncol = (size_t)ctx->T + horizon - 1;
  const double* d_th;
  const int* d_tu;
  if (int r = stage_inputs(ctx, theta, P, B, T_use, &d_th, &d_tu)) return r;
  if (int r = run_trajectory(ctx, model_kind, param_space, d_th, P, B, d_tu, horizon, rec_len)) return r;
  // outputs: one device block [preds | load1 | load2 | factors | states]
  const size_t nN = (size_t)N * ncol * B, nM = (size_t)M * ncol * B, nL = (size_t)L * ncol * B;
  YFM_HIP_CHECK(ctx->rec_P.ensure(sizeof(double) * (3 * nN + nM + nL)));
  double* d = static_cast<double*>(ctx->rec_P.p);
  yfm::PredictArgs a = predict_args(ctx, model_kind, d_th, P, B, d_tu, horizon, rec_len);
  a.preds = d;
  a.load1 = loadings_1 ? d + nN : nullptr;
  a.load2 = loadings_2 ? d + 2 * nN : nullptr;
  a.factors = d + 3 * nN;
  a.states = d + 3 * nN + nM;
  YFM_HIP_CHECK(yfm::launch_predict_emit(a));
  YFM_HIP_CHECK(hipMemcpyAsync(preds, a.preds, sizeof(double) * nN, hipMemcpyDeviceToHost, ctx->stream));
  if (loadings_1)
    YFM_HIP_CHECK(hipMemcpyAsync(loadings_1, a.load1, sizeof(double) * nN, hipMemcpyDeviceToHost, ctx->stream));
  if (loadings_2)
    YFM_HIP_CHECK(hipMemcpyAsync(loadings_2, a.load2, sizeof(double) * nN, hipMemcpyDeviceToHost, ctx->stream));
  YFM_HIP_CHECK(hipMemcpyAsync(factors, a.factors, sizeof(double) * nM, hipMemcpyDeviceToHost, ctx->stream));
  YFM_HIP_CHECK(hipMemcpyAsync(states, a.states, sizeof(double) * nL, hipMemcpyDeviceToHost, ctx->stream));
  YFM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  return YFM_OK;
}

int yfm_forecast(yfm_ctx* ctx, int model_kind, int param_space, const double* theta, int P, int B, const int* T_use,
                 int horizon, double* out) {
  if (int r = check_ctx(ctx)) return r;
  if (int r = check_batch(ctx, model_kind, param_space, P, B)) return r;
  if (horizon < 1) return set_error(YFM_EINVAL, "horizon = %d < 1", horizon);
  if (B > 0 && (!theta || !out)) return set_error(YFM_EINVAL, "null pointer argument");
  if (int r = validate_tuse(T_use, B, ctx->T)) return r;
  if (B == 0) return YFM_OK;
  const int M = state_dim(model_kind), L = gamma_dim(model_kind), N = ctx->N;
  const double* d_th;
  const int* d_tu;
  if (int r = stage_inputs(ctx, theta, P, B, T_use, &d_th, &d_tu)) return r;
  if (int r = run_trajectory(ctx, model_kind, param_space, d_th, P, B, d_tu, horizon, horizon + 1)) return r;
  const size_t n = (size_t)(M + L + N) * horizon * B;
  YFM_HIP_CHECK(ctx->rec_P.ensure(sizeof(double) * n));
  yfm::PredictArgs a = predict_args(ctx, model_kind, d_th, P, B, d_tu, horizon, horizon + 1);
  a.preds = static_cast<double*>(ctx->rec_P.p);
  YFM_HIP_CHECK(yfm::launch_forecast_emit(a));
  YFM_HIP_CHECK(hipMemcpyAsync(out, a.preds, sizeof(double) * n, hipMemcpyDeviceToHost, ctx->stream));
  YFM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  return YFM_OK;
}

int yfm_loss_array(yfm_ctx* ctx, int model_kind, int param_space, const double* theta, int P, int B,
                   const int* T_use, int K, double* mse_out) {
  if (int r = check_ctx(ctx)) return r;
  if (int r = check_batch(ctx, model_kind, param_space, P, B)) return r;
  if (K < 1) return set_error(YFM_EINVAL, "K = %d < 1", K);
  if (K > 1 && T_use) return set_error(YFM_EUNSUPPORTED, "K > 1 passes with per-candidate windows");
  if (B > 0 && (!theta || !mse_out)) return set_error(YFM_EINVAL, "null pointer argument");
  if (int r = validate_tuse(T_use, B, ctx->T)) return r;
  const int T1 = ctx->T - 1;
  if (B == 0 || T1 <= 0) return YFM_OK;
  const double* d_th;
  const int* d_tu;
  if (int r = stage_inputs(ctx, theta, P, B, T_use, &d_th, &d_tu)) return r;
  PanelView pv{static_cast<const double*>(ctx->raw.p), static_cast<const double*>(ctx->panel.p), ctx->T};
  if (K > 1) {
    // the K passes continue the filter state (filter.jl:221-242 never re-initialises):
    // filter the panel [Y[:, 1:T−1] × K, Y[:, T]] once
    const int Tk = K * T1 + 1;
    const size_t colb = sizeof(double) * ctx->N;
    YFM_HIP_CHECK(ctx->tiled_raw.ensure(colb * Tk));
    YFM_HIP_CHECK(ctx->tiled_panel.ensure(sizeof(double) * (size_t)ctx->ldp * Tk));
    char* dst = static_cast<char*>(ctx->tiled_raw.p);
    for (int k = 0; k < K; ++k)
      YFM_HIP_CHECK(hipMemcpyAsync(dst + colb * k * T1, ctx->raw.p, colb * T1, hipMemcpyDeviceToDevice, ctx->stream));
    YFM_HIP_CHECK(hipMemcpyAsync(dst + colb * K * T1, static_cast<char*>(ctx->raw.p) + colb * T1, colb,
                                 hipMemcpyDeviceToDevice, ctx->stream));
    YFM_HIP_CHECK(yfm::launch_prep_panel(static_cast<const double*>(ctx->tiled_raw.p), ctx->N, Tk, ctx->np, ctx->ldp,
                                         static_cast<double*>(ctx->tiled_panel.p), ctx->stream));
    pv = PanelView{static_cast<const double*>(ctx->tiled_raw.p), static_cast<const double*>(ctx->tiled_panel.p), Tk};
  }
  const int rec_len = pv.T - 1;
  if (int r = run_trajectory(ctx, model_kind, param_space, d_th, P, B, d_tu, 0, rec_len, &pv)) return r;
  unsigned int* cur = static_cast<unsigned int*>(ctx->flags.p) + yfm::kFlagsPerBank * ctx->bank;
  YFM_HIP_CHECK(hipMemsetAsync(cur, 0, 2 * sizeof(unsigned int), ctx->stream));
  YFM_HIP_CHECK(ctx->rec_P.ensure(sizeof(double) * (size_t)T1 * B));
  yfm::PredictArgs a = predict_args(ctx, model_kind, d_th, P, B, d_tu, 1, rec_len);
  a.preds = static_cast<double*>(ctx->rec_P.p);
  YFM_HIP_CHECK(yfm::launch_loss_array(a, static_cast<const double*>(ctx->raw.p), T1, K,
                                       cur));
  YFM_HIP_CHECK(hipMemcpyAsync(mse_out, a.preds, sizeof(double) * (size_t)T1 * B, hipMemcpyDeviceToHost, ctx->stream));
  YFM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  return YFM_OK;
}

}  // extern "C"

namespace yfm {

Workspace* workspace_create() {
  auto* w = new Workspace;
  if (w->flags.ensure(2 * yfm::kFlagsPerBank * sizeof(unsigned int)) != hipSuccess ||
      hipMemset(w->flags.p, 0, 2 * yfm::kFlagsPerBank * sizeof(unsigned int)) != hipSuccess) {
    delete w;
    return nullptr;
  }
  return w;
}

void workspace_destroy(Workspace* w) {
  if (!w) return;
  for (DevBuf* b : {&w->flags, &w->scratch, &w->scratch_dd, &w->defer, &w->scratch_fd}) b->release();
  delete w;
}

int loglik_device_ws(yfm_ctx* ctx, Workspace* ws, int kind, int space, const double* d_theta, int P, int B,
                     const int* d_T_use, double* d_out, hipStream_t s) {
  if (int r = check_ctx(ctx)) return r;
  if (int r = check_batch(ctx, kind, space, P, B)) return r;
  return launch(ctx, kind, space, d_theta, P, B, d_T_use, d_out, nullptr, nullptr, s, 0, 0, nullptr, true, ws);
}

void set_lane_share(yfm_ctx* ctx, int share) {
  if (ctx) ctx->lane_share = share > 1 ? share : 1;
}

}  // namespace yfm

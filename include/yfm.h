/*
 * yfm.h — C ABI of libyfm_hip.so: the batched Kalman-filter log-likelihood of
 * YieldFactorModels.jl on MI355X (gfx950).
 *
 * The reference has no FFI on this path; its plug-in point is Julia multiple
 * dispatch.  Each entry point below names the reference function it replaces
 * (paths relative to the reference root) — the Julia-side `@ccall` binding a
 * maintainer would add is in INTEGRATION.md.
 *
 * Conventions
 *   - All arrays are plain host (or, for *_device, device) pointers with explicit
 *     sizes.  Matrices are column-major like Julia's: the panel Y is N×T
 *     (rows = maturities, columns = months, data_management.jl:1-5) and a batch
 *     of parameter vectors Θ is P×B (candidate b is Θ[:, b], contiguous).
 *   - FP64 throughout (the reference's Float64 path, test.jl:25).
 *   - Return value: YFM_OK (0) or a negative yfm_status; yfm_last_error() then
 *     holds a thread-local message.  Numeric failures of one candidate are NOT
 *     errors: they are written into that candidate's output (see below).
 *   - A context is bound to one HIP device and is not thread-safe; use one
 *     context per host thread / per GPU.  Host-pointer calls are synchronous.
 *
 * Per-candidate numeric semantics (bitwise the reference's values)
 *   loglik_out[b] = +loglik as returned by get_loss (filter.jl:182-209):
 *     -Inf  where the reference returns -Inf (det F < 0 at t ≥ 2: DomainError in
 *           logdet, filter.jl:197-200; any non-finite loglik, filter.jl:202-204);
 *     NaN   where the reference would THROW from initialize_filter (singular
 *           I − Φ or I − Φ⊗Φ, filter.jl:4,7) — counted in n_init_throw.
 */
#ifndef YFM_H
#define YFM_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YFM_ABI_VERSION 2

typedef struct yfm_ctx yfm_ctx;

/* model_kind — create_model codes (src/model_dictionary.jl:11-16) */
enum yfm_model_kind {
  YFM_MODEL_DNS = 0,  /* "1C" / "0": DNSModel, fixed λ, M = 3, P = 20 (dns.jl) */
  YFM_MODEL_TVL = 1,  /* "TVλ" / "1": TVλDNSModel EKF, M = 4, P = 31 (tvλdns.jl) */
  YFM_MODEL_GNS5 = 2  /* extension, not in the reference: 5-factor generalised NS, M = 5, P = 48 */
};

/* param_space */
enum yfm_param_space {
  YFM_THETA_UNCONSTRAINED = 0, /* θ as compute_loss receives it (optimization.jl:10-23) */
  YFM_THETA_CONSTRAINED = 1    /* θ_c as set_params! receives it (paramoperations.jl:6-68) */
};

enum yfm_status {
  YFM_OK = 0,
  YFM_EINVAL = -1,      /* bad argument (sizes, kind, pointer) */
  YFM_EHIP = -2,        /* HIP runtime error */
  YFM_ENOPANEL = -3,    /* no panel set on this context */
  YFM_EUNSUPPORTED = -4 /* valid request this build has no kernel for */
};

/* precision — the arithmetic of the TVλ EKF (the fixed-loading models always run their FP64
 * collapsed form, whose filter contracts, with ill-conditioned-loading candidates evaluated in
 * double-double — see yfm_last_batch_deferred)
 *   YFM_PREC_CERTIFIED (default)  TVλ in double-double (~106-bit) arithmetic.  A share of TVλ
 *       candidates amplify any FP64 rounding by 1e10..1e20 over T = 600 steps, so no FP64
 *       evaluation — the reference's own dense path included — is then within 1e-9 of the
 *       exact value of filter.jl:12-80; this mode returns that value to ~1e-13 (every candidate of
 *       a 1,024-candidate config-3 sample within 1.6e-10 of a binary128 restatement, where the
 *       reference's dense FP64 path is up to 1.1e-2 from it).  ≈4× the cost of FP64.
 *   YFM_PREC_FP64  FP64 throughout, the fastest path — the reference's arithmetic class, not a
 *       certified mode: on the rounding-amplifying candidates every FP64 result, the reference's
 *       included, is rounding noise around the exact value (on the 1,024-candidate sample this mode
 *       is closer to it than the reference's dense path at the median, p99 and max — 6.7e-3 vs
 *       1.1e-2 — but either can be the closer one on a given candidate).  Off the configuration
 *       shapes its tail is wider than the reference's: on 72,947 random candidates (N 1..96, starts far
 *       from the data) p99 3.7e-9 vs 6.1e-10, 104 vs 40 above 1e-6 — the capacitance form's
 *       (v'v − u'Wu)/σ² cancels where the dense form does not.  Use YFM_PREC_CERTIFIED for
 *       results that must not depend on rounding. */
enum yfm_precision { YFM_PREC_CERTIFIED = 0, YFM_PREC_FP64 = 1 };

/* Library/ABI introspection. */
int yfm_abi_version(void);
/* Length P of θ for a model kind (kalmanbasemodel.jl:106-112 + dns.jl:15-22). */
int yfm_param_count(int model_kind);
/* State dimension M (3 DNS, 4 TVλ, 5 GNS5). */
int yfm_state_dim(int model_kind);
/* Thread-local message for the last failing call on this thread ("" if none). */
const char* yfm_last_error(void);

/* Context lifetime.  Replaces the per-model preallocated buffers of
 * KalmanBaseModel (kalmanbasemodel.jl:46-130): device buffers live in the ctx. */
yfm_ctx* yfm_create(int hip_device);
void yfm_destroy(yfm_ctx* ctx);

/* Select the TVλ arithmetic for subsequent calls on this context (default YFM_PREC_CERTIFIED).
 * The reference has no such switch: its Float64 path is YFM_PREC_FP64's arithmetic class. */
int yfm_set_precision(yfm_ctx* ctx, int precision);
int yfm_get_precision(yfm_ctx* ctx);

/* Page-locked host memory for the host-pointer entry points: θ batches and output buffers
 * allocated here are copied by DMA without a staging pass (the caller keeps the Julia/Python
 * array view; free with yfm_free_host).  NULL on failure (yfm_last_error). */
void* yfm_alloc_host(size_t bytes);
int yfm_free_host(void* p);

/* Upload the yield panel.  Y: N×T column-major (the `data` argument of get_loss,
 * filter.jl:182); maturities: N (KalmanBaseModel.maturities).  Copied; the
 * caller keeps ownership.  NaN columns are allowed (prediction-only steps). */
int yfm_set_panel(yfm_ctx* ctx, const double* Y, int N, int T, const double* maturities);

/* Batched log-likelihood — replaces B calls of
 *   compute_loss(model, data, θ_b)  (optimization.jl:10-23; loglik = -loss) when
 *   param_space = YFM_THETA_UNCONSTRAINED, or
 *   set_params!(model, θ_b); get_loss(model, data)  (filter.jl:182-209)
 *   when param_space = YFM_THETA_CONSTRAINED.
 * theta: P×B column-major.  T_use: NULL (every candidate uses all T columns) or
 * B window lengths, candidate b then evaluates get_loss(model, data[:, 1:T_use[b]])
 * (the expanding-window re-estimation of forecasting.jl:140-176), 1 ≤ T_use[b] ≤ T.
 * loglik_out: B doubles.  Synchronous. */
int yfm_loglik_batch(yfm_ctx* ctx, int model_kind, int param_space, const double* theta, int P, int B,
                     const int* T_use, double* loglik_out);

/* Same with DEVICE pointers on the caller's HIP stream (hipStream_t passed as
 * void*, NULL = default stream); asynchronous: returns after enqueueing.  For
 * pipelines that keep Θ resident in HBM (bench.py, RCCL sharding).  A context's
 * device scratch and counters serve one launch at a time: consecutive launches on
 * the same stream are ordered by the stream; a caller that moves to another stream
 * orders the two itself (hipStreamWaitEvent or a synchronisation), as for any HIP
 * work sharing buffers.  The library never touches a previous launch's stream. */
int yfm_loglik_batch_device(yfm_ctx* ctx, int model_kind, int param_space, const double* d_theta, int P, int B,
                            const int* d_T_use, double* d_loglik_out, void* hip_stream);

/* Filtered-state trajectories for parity checks: after every filter! call t
 * (t = 1..T-1), beta and P hold a_{t+1|t}, P_{t+1|t} (filter.jl:125-179).
 * beta_out: M × (T-1) × B, P_out: M × M × (T-1) × B (column-major), loglik_out: B.
 * Meant for small B (the output is O(B·T·M²)).  Synchronous. */
int yfm_filter_states(yfm_ctx* ctx, int model_kind, int param_space, const double* theta, int P, int B,
                      const int* T_use, double* beta_out, double* P_out, double* loglik_out);

/* Length L of base.gamma, the observation-driven parameters predict reports as
 * `states` (kalmanbasemodel.jl:58): 1 for DNS (dns.jl:18) and TVλ (tvλdns.jl:19,
 * never set, so zeros), 2 for the GNS5 extension. */
int yfm_gamma_dim(int model_kind);

/* Batched predict — replaces, per candidate b,
 *   set_params!(model, θ_b); predict(model, hcat(Y[:, 1:T_b], fill(NaN, N, horizon-1)))
 * (filter.jl:250-282 on the NaN padding of forecasting.jl:141/161/242); horizon = 1
 * is predict(model, Y[:, 1:T_b]).  T_b = T_use[b] (or T when T_use is NULL).
 * Outputs, column-major with ncol = T + horizon - 1 columns per candidate (candidate
 * b's columns beyond T_b + horizon - 1 are NaN):
 *   preds N×ncol×B (preds[:, j] = ŷ for observation j+1), factors M×ncol×B,
 *   states L×ncol×B (L = yfm_gamma_dim), loadings_1 / loadings_2 N×ncol×B (Z[:,2],
 *   Z[:,3]; either may be NULL).  A candidate whose initialize_filter would throw
 *   gets NaN everywhere.  Synchronous. */
int yfm_predict(yfm_ctx* ctx, int model_kind, int param_space, const double* theta, int P, int B, const int* T_use,
                int horizon, double* preds, double* factors, double* states, double* loadings_1,
                double* loadings_2);

/* Forecast blocks of the rolling-window driver (forecasting.jl:236-250):
 *   res = vcat(factors[:, end-h+1:end], states[:, end-h+1:end], preds[:, end-h+1:end])
 * of the predict call above, h = horizon.  out: (M+L+N) × h × B column-major.  This
 * is the per-task record run_forecast_window_database stores (forecasting.jl:181-184). */
int yfm_forecast(yfm_ctx* ctx, int model_kind, int param_space, const double* theta, int P, int B, const int* T_use,
                 int horizon, double* out);

/* Batched get_loss_array(model, Y[:, 1:T_b]; K) (filter.jl:211-247): mse_out (T-1)×B,
 * column b holds the T_b - 1 per-step values -‖y_t - ŷ_t‖²/N/K (entry 1 is 0, as in
 * the reference) followed by NaN.  A candidate for which the reference returns the
 * scalar -Inf (a non-finite step) gets -Inf in all its entries; NaN where
 * initialize_filter would throw.  K > 1 passes continue the filter state, as in the
 * reference; K > 1 requires T_use = NULL.  Synchronous. */
int yfm_loss_array(yfm_ctx* ctx, int model_kind, int param_space, const double* theta, int P, int B,
                   const int* T_use, int K, double* mse_out);

/* Batched estimation — replaces R calls of estimate_steps! (optimization.jl:137-312) for
 * a Kalman model with every parameter in group "1" (kalmanbasemodel.jl:150-159), i.e.
 * block-coordinate Nelder–Mead (Optim.NelderMead(), opt1: `iterations`, `g_tol`;
 * optimization.jl:442-451, :479) with the outer loop max_group_iters / |ΔLL| < tol.
 * Chain r starts from theta0[:, r] (param_space as above; the reference receives
 * constrained all_params and untransforms them) on the window Y[:, 1:T_use[r]] (or all
 * T columns when T_use is NULL).  The R chains' objective evaluations are batched into
 * one device launch per round.  Outputs: theta_c_out P×R = transform_params(best_p)
 * (the reference's returned params), p_out P×R unconstrained optimum (or NULL), init_c_out P×R
 * (or NULL) = transform_params of the sanitised, ×0.95-rescaled start (the reference's returned
 * init_p, optimization.jl:157-184, :298-302), ll_out R
 * (the reference's returned ll), status_out R (or NULL): 0 ok, 1 the reference would
 * throw (NaN outputs), 2 aborted after the first group iteration (parameters kept);
 * n_evals_out (or NULL): objective evaluations performed.  Synchronous. */
int yfm_estimate(yfm_ctx* ctx, int model_kind, int param_space, const double* theta0, int P, int R,
                 const int* T_use, int iterations, double g_tol, int max_group_iters, double tol,
                 double* theta_c_out, double* p_out, double* init_c_out, double* ll_out, int* status_out,
                 long long* n_evals_out);

/* Counters of the last completed batch on this ctx: candidates where the
 * reference would have thrown (NaN outputs) and candidates returning -Inf.
 * For yfm_loglik_batch_device, synchronise the stream first. */
int yfm_last_batch_flags(yfm_ctx* ctx, long long* n_init_throw, long long* n_neg_inf);

/* Candidates of the last completed batch on this ctx that the fixed-loading models (DNS, GNS5)
 * evaluated on the double-double capacitance path instead of the FP64 collapsed form: an
 * ill-conditioned loading Gram matrix (κ₁(Z'Z) ≥ 1e6), a singular one, or fewer maturities than
 * states.  Same filter!/get_loss semantics (filter.jl:125-209); reported for auditing the cost
 * and accuracy split (0 for TVλ).  For yfm_loglik_batch_device, synchronise the stream first. */
int yfm_last_batch_deferred(yfm_ctx* ctx, long long* n_deferred);

/* Wave-steps of the last batch that ran in the DNS / GNS5 kernel's frozen-covariance steady state (64
 * filter steps each: the mean update only at the converged P — DNS with the factors of S = P + R
 * cached, GNS5 refactoring the constant S — DESIGN.md §3.1).  The covariance recursion of filter.jl:158-176 does not depend on the data when the
 * loadings are fixed; a candidate freezes its P once the change per step is at the rounding level, at a
 * step that depends on its own θ only.  YFM_DNS_STEADY=0 in the environment disables it.  0 for the
 * other models, for trajectories and for panels shorter than 80 columns (full recursion there). */
int yfm_last_batch_steady(yfm_ctx* ctx, long long* steady_wave_steps);

#ifdef __cplusplus
}
#endif
#endif /* YFM_H */

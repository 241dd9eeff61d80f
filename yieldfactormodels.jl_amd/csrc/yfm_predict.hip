// yfm_predict.hip — the trajectory outputs of the Kalman filter, built from the state
// trajectory that the filter kernels record in trajectory mode (LaunchArgs::horizon,
// rec_len).  Restates, per candidate θ_b:
//   predict          src/models/kalman/filter.jl:250-282   (preds, factors, states,
//                    factor_loadings_1/2; the final NaN step gives the last column)
//   forecast blocks  src/forecasting.jl:236-250 (res = [factors; states; preds] over the
//                    last `horizon` columns of predict on hcat(data[:,1:task], NaN×(h−1)))
//   get_loss_array   src/models/kalman/filter.jl:211-247   (per-step −‖y_t − ŷ_t‖²/N/K)
//
// Alignment (A_j = the state after filter! step j, 1-based, as recorded in slot j−1):
// filter! on column t first forms ŷ = Z(β)β from the state BEFORE the step, so
//   preds[:, j] = Z(A_j) A_j,   factors[:, j] = A_{j+1},   j = 1 .. n
// for n = T_b + horizon − 1 padded columns.  Column j therefore reads slots j−1 and j of
// the trajectory.  Loadings: fixed per candidate (DNS / GNS5, from γ), or from the
// predicted β₄ of the same state (TVλ, tvλdns.jl:53-64, called at filter.jl:14/32).
//
// These kernels write the outputs (HBM-bound, one thread per output element for the
// N-sized arrays); the filter recursion itself stays in yfm_kernels.hip / yfm_tvl.hip.
#include "../../include/yfm.h"
#include "yfm_device.hpp"
#include "yfm_internal.hpp"

namespace yfm {

namespace {

// dns.jl:51-65 / tvλdns.jl:53-64 for one maturity, in the filter kernels' arithmetic
__device__ __forceinline__ void ns_loadings(double lam, double m, double& s, double& c) {
  const double tau = lam * m;
  const double z = exp(-tau);
  s = (1.0 - z) / tau;
  c = s - z;
}

// ŷ_i = (Z(A) A)_i and the two loading columns the reference reports (Z[:,2], Z[:,3])
__device__ __forceinline__ void fitted(int kind, const double* __restrict__ A, const double* __restrict__ th,
                                       double m, double& pred, double& l1, double& l2) {
  if (kind == YFM_MODEL_TVL) {
    ns_loadings(1e-2 + exp(A[3]), m, l1, l2);  // λ from the predicted β₄
    pred = fma(A[2], l2, fma(A[1], l1, A[0]));  // Z[:,1:3] β[1:3] (filter.jl:15, :33)
  } else {
    ns_loadings(1e-2 + exp(th[0]), m, l1, l2);
    pred = fma(A[2], l2, fma(A[1], l1, A[0]));
    if (kind == YFM_MODEL_GNS5) {
      double s2, c2;
      ns_loadings(1e-2 + exp(th[1]), m, s2, c2);
      pred = fma(A[4], c2, fma(A[3], s2, pred));
    }
  }
}

constexpr unsigned long long kNaNBits = 0x7ff8000000000000ull;

__device__ __forceinline__ double qnan() { return __longlong_as_double((long long)kNaNBits); }

// One thread per (candidate b, column j, maturity i) of predict's N-row outputs; the
// i = 0 thread of each (b, j) also writes the M factors and the L states.
__global__ __launch_bounds__(256) void predict_emit_kernel(
    int kind, int M, int L, int N, int ncol, int horizon, int B, int P, const double* __restrict__ theta,
    const double* __restrict__ mats, const int* __restrict__ T_use, int T, const double* __restrict__ rec,
    int rec_len, const unsigned char* __restrict__ init_bad, double* __restrict__ preds,
    double* __restrict__ factors, double* __restrict__ states, double* __restrict__ load1,
    double* __restrict__ load2) {
  const size_t total = (size_t)B * ncol * N;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(e % N);
    const size_t bj = e / N;
    const int j = (int)(bj % ncol);
    const int b = (int)(bj / ncol);
    const int nb = (T_use ? T_use[b] : T) + horizon - 1;  // padded data columns of candidate b
    const double* th = theta + (size_t)b * P;
    double pr = qnan(), l1 = qnan(), l2 = qnan();
    const bool valid = j < nb && !init_bad[b];
    const double* A = rec + ((size_t)b * rec_len + j) * M;  // slot j = A_{j+1}
    if (valid) fitted(kind, A, th, mats[i], pr, l1, l2);
    preds[e] = pr;
    if (load1) load1[e] = l1;
    if (load2) load2[e] = l2;
    if (i == 0) {
      const double* An = A + M;  // slot j + 1 = A_{j+2}
      for (int k = 0; k < M; ++k) factors[bj * M + k] = valid ? An[k] : qnan();
      for (int l = 0; l < L; ++l) {
        const double g = (kind == YFM_MODEL_TVL) ? 0.0 : th[l];  // base.gamma (TVλ: never set, zeros)
        states[bj * L + l] = valid ? g : qnan();
      }
    }
  }
}

// forecasting.jl:236-250: res = [factors; states; preds] over the last h columns, one
// (M + L + N) × h block per candidate.  The trajectory holds the last h + 1 states.
__global__ __launch_bounds__(256) void forecast_emit_kernel(int kind, int M, int L, int N, int h, int B, int P,
                                                            const double* __restrict__ theta,
                                                            const double* __restrict__ mats,
                                                            const double* __restrict__ rec,
                                                            const unsigned char* __restrict__ init_bad,
                                                            double* __restrict__ out) {
  const int R = M + L + N;
  const size_t total = (size_t)B * h * N;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(e % N);
    const size_t bk = e / N;
    const int k = (int)(bk % h);
    const int b = (int)(bk / h);
    const double* th = theta + (size_t)b * P;
    const double* A = rec + ((size_t)b * (h + 1) + k) * M;
    const bool valid = !init_bad[b];
    double pr = qnan(), l1, l2;
    if (valid) fitted(kind, A, th, mats[i], pr, l1, l2);
    double* o = out + bk * R;
    o[M + L + i] = pr;
    if (i == 0) {
      for (int q = 0; q < M; ++q) o[q] = valid ? A[M + q] : qnan();
      for (int l = 0; l < L; ++l) o[M + l] = valid ? ((kind == YFM_MODEL_TVL) ? 0.0 : th[l]) : qnan();
    }
  }
}

// get_loss_array (filter.jl:211-247): out[b, t] for t = 0 .. T−2 (Julia t = 1 .. nobs−1),
// accumulated over `passes` passes whose states continue (the reference does not
// re-initialise between its K passes).  Step s = k(T−1) + t of the recorded trajectory
// (panel tiled K times) is pass k, column t; ŷ uses the state before the step, slot s − 1.
// Julia t = 1 of every pass is never accumulated (:230), so slot −1 (β₀) is never needed.
__global__ __launch_bounds__(256) void loss_array_kernel(int kind, int M, int N, int T1, int passes, int B, int P,
                                                         const double* __restrict__ theta,
                                                         const double* __restrict__ mats,
                                                         const double* __restrict__ Y,  // N × T column-major
                                                         const int* __restrict__ T_use,
                                                         const double* __restrict__ rec, int rec_len,
                                                         double* __restrict__ out) {
  const size_t total = (size_t)B * T1;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int t = (int)(e % T1);
    const int b = (int)(e / T1);
    const int nb = T_use ? T_use[b] - 1 : T1;  // steps of candidate b (its window's nobs − 1)
    const double* th = theta + (size_t)b * P;
    double acc = 0.0;
    if (t >= nb) {
      acc = qnan();
    } else if (t >= 1) {
      const double* y = Y + (size_t)t * N;
      for (int k = 0; k < passes; ++k) {
        const double* A = rec + ((size_t)b * rec_len + (size_t)k * nb + t - 1) * M;
        double vv = 0.0;
        for (int i = 0; i < N; ++i) {
          double pr, l1, l2;
          fitted(kind, A, th, mats[i], pr, l1, l2);
          const double v = y[i] - pr;
          vv = fma(v, v, vv);
        }
        acc -= vv;  // mse[t] -= dot(v, v)  (:231)
      }
      acc = acc / (double)N / (double)passes;  // :245
    }
    out[e] = acc;
  }
}

// a non-finite mse[t] makes get_loss_array return −Inf (:234-236): the whole row becomes −Inf
__global__ __launch_bounds__(256) void loss_array_finish_kernel(int T1, int B, const int* __restrict__ T_use,
                                                                const unsigned char* __restrict__ init_bad,
                                                                double* __restrict__ out,
                                                                unsigned int* __restrict__ flags) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int nb = T_use ? T_use[b] - 1 : T1;
  double* row = out + (size_t)b * T1;
  if (init_bad[b]) {  // the reference throws from initialize_filter
    for (int t = 0; t < T1; ++t) row[t] = qnan();
    atomicAdd(&flags[0], 1u);
    return;
  }
  bool bad = false;
  for (int t = 0; t < nb; ++t) bad = bad || !isfinite(row[t]);
  if (bad) {
    for (int t = 0; t < nb; ++t) row[t] = -__builtin_inf();
    atomicAdd(&flags[1], 1u);
  }
}

// initialize_filter threw ⇔ the loglik kernel wrote NaN; mark those candidates
__global__ void init_bad_kernel(const double* __restrict__ ll, int B, unsigned char* __restrict__ bad) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) bad[b] = ll[b] != ll[b];
}

int grid_for(size_t work) {
  size_t g = (work + 255) / 256;
  return (int)(g < 16384 ? (g > 0 ? g : 1) : 16384);
}

}  // namespace

hipError_t launch_init_bad(const double* ll, int B, unsigned char* bad, hipStream_t s) {
  hipLaunchKernelGGL(init_bad_kernel, dim3((B + 255) / 256), dim3(256), 0, s, ll, B, bad);
  return hipGetLastError();
}

hipError_t launch_predict_emit(const PredictArgs& a) {
  hipLaunchKernelGGL(predict_emit_kernel, dim3(grid_for((size_t)a.B * a.ncol * a.N)), dim3(256), 0, a.stream, a.kind,
                     a.M, a.L, a.N, a.ncol, a.horizon, a.B, a.P, a.theta, a.mats, a.T_use, a.T, a.rec, a.rec_len,
                     a.init_bad, a.preds, a.factors, a.states, a.load1, a.load2);
  return hipGetLastError();
}

hipError_t launch_forecast_emit(const PredictArgs& a) {
  hipLaunchKernelGGL(forecast_emit_kernel, dim3(grid_for((size_t)a.B * a.horizon * a.N)), dim3(256), 0, a.stream,
                     a.kind, a.M, a.L, a.N, a.horizon, a.B, a.P, a.theta, a.mats, a.rec, a.init_bad, a.preds);
  return hipGetLastError();
}

hipError_t launch_loss_array(const PredictArgs& a, const double* Y, int T1, int passes, unsigned int* flags) {
  hipLaunchKernelGGL(loss_array_kernel, dim3(grid_for((size_t)a.B * T1)), dim3(256), 0, a.stream, a.kind, a.M, a.N,
                     T1, passes, a.B, a.P, a.theta, a.mats, Y, a.T_use, a.rec, a.rec_len, a.preds);
  hipLaunchKernelGGL(loss_array_finish_kernel, dim3((a.B + 255) / 256), dim3(256), 0, a.stream, T1, a.B, a.T_use,
                     a.init_bad, a.preds, flags);
  return hipGetLastError();
}

}  // namespace yfm

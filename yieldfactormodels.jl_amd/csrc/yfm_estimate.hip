// yfm_estimate.hip — batched estimation driver: R independent estimate_steps! chains
// (one per estimation window / start) whose objective evaluations are gathered, round by
// round, into ONE batched log-likelihood launch on the device (yfm_loglik_batch).
//
// Restates, per chain (reference paths relative to the reference root):
//   estimate_steps!   src/optimization.jl:137-312 for a Kalman model, all parameters in
//                     group "1" (kalmanbasemodel.jl:150-159): untransform + sanitize
//                     (:157-162, :422-432), ×0.95 rescaling of a non-finite start
//                     (:173-184), outer loop max_group_iters / |ΔLL| < tol (:218-281),
//                     rethrow on iteration 1 / abort later (:249-257), transform (:301).
//   Optim.NelderMead  with opt1 (iterations = 500, g_tol = 1e-6; optimization.jl:442-451,
//                     :479).  Optim.jl 1.13 (Project.toml:42) is not vendored in the
//                     reference; its published algorithm (adaptive parameters, affine
//                     simplexer, reflection / expansion / contractions / shrink, nm_x
//                     stopping rule, centroid-vs-best minimizer) is restated here and in
//                     oracle/optim_nm.py, against which this file is tested bit for bit.
//
// MI355X mapping: the chains are independent, so every round packs the points all
// chains need into one batch and evaluates it with one kernel launch.  A Nelder–Mead
// iteration needs the reflection and then, depending on it, one of expansion / outside
// contraction / inside contraction: all four are functions of (centroid, worst vertex),
// so one round evaluates them speculatively and the chain then takes exactly the
// reference's branch (unused values are discarded, including their failures).  A shrink
// costs one extra round.  The arithmetic of the simplex updates follows Optim's
// operation order with FP contraction off, so the chain is bitwise reproducible.
//
// Speculation tree (YFM_NM_SPEC = node budget per chain and round, default 16; 1 = none):
// besides its iteration's four trial points, a round evaluates the trial points of later
// iterations for the ways the earlier ones can end without a shrink — which trial point is
// accepted and which vertex is then the worst (see build_tree).  Nodes are picked best-first by
// the probability that the chain reaches them, estimated from the chain's own history of outcome
// transitions.  When the real outcome of an iteration is known, the chain's next iteration is
// the speculated node with the same simplex (same vertices, same worst index, so the same
// arithmetic): its values are consumed at once and it costs no round; the walk continues down
// the tree until an outcome was not speculated.  The chain's sequence of states, and so its
// result, is bitwise that of one iteration per round; n_evals counts the evaluations the chain
// consumed (as without speculation).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "../../include/yfm.h"
#include "yfm_internal.hpp"
#include "yfm_nm.hpp"

namespace {

using namespace yfm_nm;

// Page-locked host staging for the per-round batch: the runtime DMAs straight from it
// instead of bouncing pageable memory through its own buffer (one round trip per round).
struct PinnedBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    const size_t want = std::max(bytes, cap * 2);
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) cap = want;
    return e;
  }
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
};

enum Code { ID = 0, POS = 1, R11 = 2 };


// transform vectors: kalmanbasemodel.jl:74-120 (+ dns.jl:15-22 one leading γ; GNS5 two)
std::vector<int> transform_codes(int kind) {
  const int M = yfm_state_dim(kind);
  const int lead = kind == YFM_MODEL_DNS ? 1 : kind == YFM_MODEL_GNS5 ? 2 : 0;
  std::vector<int> c(lead, ID);
  c.push_back(POS);  // σ²
  for (int i = 0; i < M; ++i)
    for (int j = 0; j <= i; ++j) c.push_back(j == i ? POS : ID);  // U by column, diag exp
  for (int i = 0; i < M; ++i) c.push_back(ID);                   // δ
  for (int i = 0; i < M; ++i)
    for (int j = 0; j < M; ++j) c.push_back(i == j ? R11 : ID);  // Φ row-major
  return c;
}

// transformations.jl:2-26
double to_constrained(int code, double x) {
  if (code == POS) return std::exp(x);
  if (code == R11) {
    const double y = std::exp(x);
    return 2.0 * y / (1.0 + y) - 1.0;
  }
  return x;
}
double to_unconstrained(int code, double x) {
  if (code == POS) return std::log(x);
  if (code == R11) return std::log1p(x) - std::log1p(-x);
  return x;
}

// Minimal fork-join pool for the per-round host work (chains are independent).
//
// Round protocol (no item can run twice or leak into the next round):
//   run():   with no round open and no worker inside one, write the round's parameters, then
//            open it (open_ = its generation, seq_cst); drain; wait until every item is done;
//            close it (open_ = 0); wait until no worker is inside it (active_ == 0).
//   worker:  active_ += 1, THEN read open_ (both seq_cst); only a worker that sees the round
//            open touches its parameters; active_ −= 1 when it leaves.
// A worker that registers after run() saw active_ == 0 reads open_ after that point in the
// single total order, so it sees 0 (and leaves without reading anything) or a later round whose
// parameters were written before that round was opened.
class Pool {
 public:
  explicit Pool(int n) {
    for (int i = 1; i < n; ++i) th_.emplace_back([this] { worker(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
      stop_a_.store(true);
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // f(i) for i in [0, n), items handed out in chunks; returns when all are done and every worker
  // has left the round
  template <class F>
  void run(int n, int chunk, F&& f) {
    if (th_.empty() || n <= chunk) {
      for (int i = 0; i < n; ++i) f(i);
      return;
    }
    std::function<void(int)> job = [&](int i) { f(i); };
    bool wake;
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = &job;
      n_ = n;
      chunk_ = chunk;
      next_.store(0);
      done_.store(0);
      gen_ = gen_ == 0x7fffffff ? 1 : gen_ + 1;
      open_.store(gen_);
      wake = sleepers_ > 0;
    }
    if (wake) cv_.notify_all();
    drain();
    while (done_.load() < n) __builtin_ia32_pause();
    open_.store(0);
    while (active_.load() != 0) __builtin_ia32_pause();
    std::lock_guard<std::mutex> g(m_);
    job_ = nullptr;
  }

 private:
  void drain() {
    for (;;) {
      const int i0 = next_.fetch_add(chunk_);
      if (i0 >= n_) return;
      const int i1 = std::min(n_, i0 + chunk_);
      for (int i = i0; i < i1; ++i) (*job_)(i);
      done_.fetch_add(i1 - i0);
    }
  }
  // Rounds come every few hundred µs: a worker spins for the next one (a futex wake-up costs tens
  // of µs per thread) and only sleeps after 2 ms without work.
  void worker() {
    int seen = 0;
    for (;;) {
      const auto t0 = std::chrono::steady_clock::now();
      for (int k = 0; (open_.load() == 0 || open_.load() == seen) && !stop_a_.load(); ++k) {
        __builtin_ia32_pause();
        if ((k & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
      }
      {
        std::unique_lock<std::mutex> lk(m_);
        auto idle = [&] {
          const int o = open_.load();
          return o == 0 || o == seen;
        };
        if (!stop_ && idle()) {
          ++sleepers_;
          cv_.wait(lk, [&] { return stop_ || !idle(); });
          --sleepers_;
        }
        if (stop_) return;
      }
      active_.fetch_add(1);
      const int g = open_.load();
      if (g != 0 && g != seen) {
        seen = g;
        drain();
      }
      active_.fetch_sub(1);
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_;
  std::function<void(int)>* job_ = nullptr;
  int n_ = 0, chunk_ = 1, gen_ = 0, sleepers_ = 0;
  bool stop_ = false;
  std::atomic<int> next_{0}, done_{0}, open_{0}, active_{0};
  std::atomic<bool> stop_a_{false};
};

}  // namespace

extern "C" int yfm_estimate(yfm_ctx* ctx, int model_kind, int param_space, const double* theta0, int P, int R,
                            const int* T_use, int iterations, double g_tol, int max_group_iters, double tol,
                            double* theta_c_out, double* p_out, double* init_c_out, double* ll_out,
                            int* status_out, long long* n_evals_out) {
  if (!ctx) return yfm::api_error(YFM_EINVAL, "null context");
  if (yfm_param_count(model_kind) < 0) return yfm::api_error(YFM_EINVAL, "unknown model_kind");
  if (P != yfm_param_count(model_kind)) return yfm::api_error(YFM_EINVAL, "P does not match model_kind");
  if (param_space != YFM_THETA_UNCONSTRAINED && param_space != YFM_THETA_CONSTRAINED)
    return yfm::api_error(YFM_EINVAL, "unknown param_space");
  if (R < 0 || iterations < 0 || max_group_iters < 1)
    return yfm::api_error(YFM_EINVAL, "R, iterations must be >= 0 and max_group_iters >= 1");
  if (R == 0) return YFM_OK;
  if (!theta0 || !theta_c_out || !ll_out) return yfm::api_error(YFM_EINVAL, "null pointer argument");
  const int Tp = yfm::panel_T(ctx);
  if (Tp <= 0) return yfm::api_error(YFM_ENOPANEL, "no panel: call yfm_set_panel first");
  // the estimator's group streams share the context's buffers with any earlier launch on a caller's stream
  if (yfm::settle_foreign_launch(ctx) != hipSuccess) return yfm::api_error(YFM_EHIP, "device synchronisation failed");
  if (T_use)
    for (int r = 0; r < R; ++r)
      if (T_use[r] < 1 || T_use[r] > Tp) return yfm::api_error(YFM_EINVAL, "T_use outside [1, T]");
  const std::vector<int> codes = transform_codes(model_kind);
  std::vector<Chain> chains(R);
  for (int r = 0; r < R; ++r) {
    Chain& c = chains[r];
    c.n = P;
    c.window = T_use ? T_use[r] : 0;
    c.p.resize(P);
    for (int i = 0; i < P; ++i) {
      double x = theta0[(size_t)r * P + i];
      if (param_space == YFM_THETA_CONSTRAINED) x = to_unconstrained(codes[i], x);
      c.p[i] = std::isfinite(x) ? x : 0.0;  // _sanitize_parameters (optimization.jl:422-432)
    }
  }
  int spec_nodes = 16;
  if (const char* e = std::getenv("YFM_NM_SPEC")) spec_nodes = std::max(1, std::min(kMaxNodes, std::atoi(e)));
  const bool stats = std::getenv("YFM_EST_STATS") != nullptr;
  // Every chain owns a fixed slot of SLOT points in the round's batch (its requests, then its
  // speculated points; the rest of the slot keeps earlier values and its results are ignored),
  // so each chain's host work — consume the last results, prepare, write the slot — runs in
  // parallel, straight into page-locked memory, and T_use is written once.
  const int SLOT = std::max(4 * spec_nodes, P + 1);
  if (SLOT > kMaxSlot) return yfm::api_error(YFM_EINVAL, "too many parameters for the estimation driver");
  const int B = R * SLOT;
  PinnedBuf pin_th, pin_tu, pin_out;
  if (pin_th.ensure(sizeof(double) * (size_t)B * P) != hipSuccess ||
      pin_out.ensure(sizeof(double) * (size_t)B) != hipSuccess ||
      (T_use && pin_tu.ensure(sizeof(int) * (size_t)B) != hipSuccess))
    return yfm::api_error(YFM_EHIP, "hipHostMalloc failed for the estimation batch");
  double* th = static_cast<double*>(pin_th.p);
  double* out = static_cast<double*>(pin_out.p);
  // Zero-copy rounds (default): the filter kernel reads θ from, and writes the logliks to, the
  // page-locked buffers themselves — no DMA transfers to wait for between the host bookkeeping and
  // the launch (θ is read once per lane, the loglik written once).
  bool zero_copy = true;
  if (const char* e = std::getenv("YFM_EST_ZEROCOPY")) zero_copy = std::atoi(e) != 0;
  double *map_th = nullptr, *map_out = nullptr;
  if (zero_copy && (hipHostGetDevicePointer(reinterpret_cast<void**>(&map_th), th, 0) != hipSuccess ||
                    hipHostGetDevicePointer(reinterpret_cast<void**>(&map_out), out, 0) != hipSuccess))
    zero_copy = false;
  std::memset(th, 0, sizeof(double) * (size_t)B * P);
  if (T_use)
    for (int r = 0; r < R; ++r) std::fill_n(static_cast<int*>(pin_tu.p) + (size_t)r * SLOT, SLOT, T_use[r]);
  // Chains are split into G groups, each with its own stream and launch workspace: while one
  // group's batch is on the device, the host consumes the other group's results and prepares its
  // next round, and the two groups' filters run concurrently (each fills a small part of the chip),
  // so a round costs one filter latency instead of filter + host bookkeeping + transfers.
  int G = R >= 32 ? 2 : 1;
  if (const char* e = std::getenv("YFM_EST_GROUPS")) G = std::max(1, std::min(kMaxGroups, std::atoi(e)));
  // device-side batch: θ uploaded per round on each group's own stream, T_use once
  hipStream_t sts[kMaxGroups] = {};
  yfm::Workspace* wss[kMaxGroups] = {};  // group 0 uses the context's own buffers
  double *d_th = nullptr, *d_out = nullptr;
  int* d_tu = nullptr;
  struct Release {
    hipStream_t (&s)[kMaxGroups];
    yfm::Workspace* (&w)[kMaxGroups];
    double*& a;
    double*& b;
    int*& c;
    ~Release() {
      for (hipStream_t x : s)
        if (x) (void)hipStreamSynchronize(x);
      if (a) (void)hipFree(a);
      if (b) (void)hipFree(b);
      if (c) (void)hipFree(c);
      for (hipStream_t x : s)
        if (x) (void)hipStreamDestroy(x);
      for (yfm::Workspace* x : w) yfm::workspace_destroy(x);
    }
  } release{sts, wss, d_th, d_out, d_tu};
  // the G groups' launches run side by side: each group's TVλ launch is sized for its share of the device
  struct Share {
    yfm_ctx* c;
    ~Share() { yfm::set_lane_share(c, 1); }
  } share_reset{ctx};
  yfm::set_lane_share(ctx, G);
  for (int g = 0; g < G; ++g)
    if (hipStreamCreateWithFlags(&sts[g], hipStreamNonBlocking) != hipSuccess)
      return yfm::api_error(YFM_EHIP, "stream creation failed for the estimation batch");
  for (int g = 1; g < G; ++g)
    if (!(wss[g] = yfm::workspace_create()))
      return yfm::api_error(YFM_EHIP, "workspace allocation failed for the estimation batch");
  if (hipMalloc(&d_th, sizeof(double) * (size_t)B * P) != hipSuccess ||
      hipMalloc(&d_out, sizeof(double) * (size_t)B) != hipSuccess ||
      (T_use && hipMalloc(&d_tu, sizeof(int) * (size_t)B) != hipSuccess))
    return yfm::api_error(YFM_EHIP, "device allocation failed for the estimation batch");
  if (T_use && hipMemcpy(d_tu, pin_tu.p, sizeof(int) * (size_t)B, hipMemcpyHostToDevice) != hipSuccess)
    return yfm::api_error(YFM_EHIP, "T_use upload failed");
  int nthreads = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  if (const char* e = std::getenv("YFM_EST_THREADS")) nthreads = std::max(1, std::atoi(e));
  Pool pool(std::min(nthreads, std::max(1, R / (4 * G))));
  std::atomic<int> active{0};
  std::atomic<int> last_active{-1};  // highest chain index of the group that requested points this round
  long long device_evals = 0, rounds = 0;
  double t_host = 0.0, t_dev = 0.0;
  using clk = std::chrono::steady_clock;
  std::atomic<long long> ns_consume{0}, ns_prepare{0}, ns_copy{0};  // host time split (YFM_EST_STATS)
  auto host_step = [&](int r) {
    Chain& c = chains[r];
    const auto h0 = stats ? clk::now() : clk::time_point();
    if (c.n_req > 0) {  // the results of this chain's slot from the last round
      double f[kMaxSlot];
      const int nv = c.nodes.empty() ? c.n_req : 4 * (int)c.nodes.size();
      for (int k = 0; k < nv; ++k) f[k] = -out[(size_t)r * SLOT + k];  // compute_loss = −loglik (optimization.jl:22)
      absorb(c, f, iterations, max_group_iters, tol, g_tol);
    }
    const auto h1 = stats ? clk::now() : clk::time_point();
    prepare(c, iterations, spec_nodes);
    const auto h2 = stats ? clk::now() : clk::time_point();
    if (c.n_req > 0) {
      active.fetch_add(1, std::memory_order_relaxed);
      for (int m = last_active.load(std::memory_order_relaxed); m < r;)
        if (last_active.compare_exchange_weak(m, r, std::memory_order_relaxed)) break;
      double* slot = th + (size_t)r * SLOT * P;
      if (c.nodes.empty())
        std::memcpy(slot, c.trial.data(), sizeof(double) * c.trial.size());
      else
        std::memcpy(slot, c.pts.data(), sizeof(double) * c.nodes.size() * 4 * (size_t)P);
    }
    if (stats) {
      const auto h3 = clk::now();
      ns_consume += std::chrono::duration_cast<std::chrono::nanoseconds>(h1 - h0).count();
      ns_prepare += std::chrono::duration_cast<std::chrono::nanoseconds>(h2 - h1).count();
      ns_copy += std::chrono::duration_cast<std::chrono::nanoseconds>(h3 - h2).count();
    }
  };
  // group g: chains [r0[g], r0[g + 1]), slots [r0[g]·SLOT, r0[g + 1]·SLOT) of every buffer
  int r0[kMaxGroups + 1];
  for (int g = 0; g <= G; ++g) r0[g] = (int)((long long)R * g / G);
  bool pending[kMaxGroups] = {};
  // launch extent per group: up to the last chain that requested points (finished chains at the
  // end of a group cost no lanes; the slots of finished chains inside it are still evaluated)
  int r_end[kMaxGroups] = {};
  auto host_group = [&](int g) {
    active.store(0);
    last_active.store(-1);
    pool.run(r0[g + 1] - r0[g], 2, [&](int i) { host_step(r0[g] + i); });
    r_end[g] = last_active.load() + 1;
    return active.load() > 0;
  };
  auto submit = [&](int g) -> int {
    const size_t o = (size_t)r0[g] * SLOT;
    const int Bg = (r_end[g] - r0[g]) * SLOT;
    if (zero_copy) {
      const int rc = yfm::loglik_device_ws(ctx, wss[g], model_kind, YFM_THETA_UNCONSTRAINED, map_th + o * P, P, Bg,
                                           d_tu ? d_tu + o : nullptr, map_out + o, sts[g]);
      if (rc != YFM_OK) return rc;
      device_evals += Bg;
      ++rounds;
      return YFM_OK;
    }
    if (hipMemcpyAsync(d_th + o * P, th + o * P, sizeof(double) * (size_t)Bg * P, hipMemcpyHostToDevice, sts[g]) !=
        hipSuccess)
      return yfm::api_error(YFM_EHIP, "θ upload failed");
    const int rc = yfm::loglik_device_ws(ctx, wss[g], model_kind, YFM_THETA_UNCONSTRAINED, d_th + o * P, P, Bg,
                                         d_tu ? d_tu + o : nullptr, d_out + o, sts[g]);
    if (rc != YFM_OK) return rc;
    if (hipMemcpyAsync(out + o, d_out + o, sizeof(double) * (size_t)Bg, hipMemcpyDeviceToHost, sts[g]) != hipSuccess)
      return yfm::api_error(YFM_EHIP, "loglik download failed");
    device_evals += Bg;
    ++rounds;
    return YFM_OK;
  };
  for (int g = 0; g < G; ++g) {
    const auto t0 = clk::now();
    pending[g] = host_group(g);
    t_host += std::chrono::duration<double>(clk::now() - t0).count();
    if (pending[g])
      if (int rc = submit(g)) return rc;
  }
  for (bool any = true; any;) {
    any = false;
    for (int g = 0; g < G; ++g) {
      if (!pending[g]) continue;
      const auto t0 = clk::now();
      if (hipStreamSynchronize(sts[g]) != hipSuccess) return yfm::api_error(YFM_EHIP, "estimation round failed");
      const auto t1 = clk::now();
      pending[g] = host_group(g);
      t_dev += std::chrono::duration<double>(t1 - t0).count();
      t_host += std::chrono::duration<double>(clk::now() - t1).count();
      if (pending[g])
        if (int rc = submit(g)) return rc;
      any = any || pending[g];
    }
  }
  rounds = (rounds + G - 1) / G;  // rounds per group (each group's chains see one launch per round)
  long long evals = 0;
  long long hits = 0;
  for (const Chain& c : chains) {
    evals += c.used;
    hits += c.spec_hits;
  }
  if (stats) {
    std::fprintf(stderr, "yfm_estimate: %lld rounds, %lld chain evaluations, %lld device evaluations, %lld "
                 "speculated iterations used; host %.3f s, waiting on the device %.3f s (%d groups)\n", rounds, evals,
                 device_evals, hits, t_host, t_dev, G);
    long long tr[8][8] = {}, dh[8] = {}, rc[2] = {};
    for (const Chain& c : chains) {
      for (int a = 0; a < 8; ++a) {
        dh[a] += c.depth_hist[a];
        for (int b = 0; b < 8; ++b) tr[a][b] += c.trans[a][b];
      }
      rc[0] += c.recent[0];
      rc[1] += c.recent[1];
    }
    std::fprintf(stderr, "yfm_estimate: host thread time: consume + tree walk %.3f s, prepare %.3f s, slot copy %.3f s "
                 "(%d threads)\n", ns_consume.load() * 1e-9, ns_prepare.load() * 1e-9, ns_copy.load() * 1e-9,
                 std::min(nthreads, std::max(1, R / (4 * G))));
    std::fprintf(stderr, "yfm_estimate: %d tree nodes per round; iterations per NM round:", spec_nodes);
    for (int a = 1; a < 8; ++a) std::fprintf(stderr, " %d:%lld", a, dh[a]);
    std::fprintf(stderr, "; worst = previously replaced vertex in %lld of %lld non-new outcomes\n", rc[0], rc[1]);
    std::fprintf(stderr, "yfm_estimate: iteration outcome transitions (row: previous, col: next; "
                 "R E O O* I I* S, * = new vertex is the worst; row 7 = first)\n");
    for (int a = 0; a < 8; ++a) {
      std::fprintf(stderr, "  %d:", a);
      for (int b = 0; b < 7; ++b) std::fprintf(stderr, " %9lld", tr[a][b]);
      std::fprintf(stderr, "\n");
    }
  }
  for (int r = 0; r < R; ++r) {
    const Chain& c = chains[r];
    const bool ok = c.status != 1;
    for (int i = 0; i < P; ++i) {
      theta_c_out[(size_t)r * P + i] = ok ? to_constrained(codes[i], c.p[i]) : NAN;
      if (p_out) p_out[(size_t)r * P + i] = c.p[i];
      if (init_c_out)
        init_c_out[(size_t)r * P + i] = (ok && !c.start.empty()) ? to_constrained(codes[i], c.start[i]) : NAN;
    }
    ll_out[r] = ok ? c.prev_ll : NAN;
    if (status_out) status_out[r] = c.status;
  }
  if (n_evals_out) *n_evals_out = evals;
  return YFM_OK;
}

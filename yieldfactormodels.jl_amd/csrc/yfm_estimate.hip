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

namespace {

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

constexpr int kMaxSlot = 128;  // points per chain and round (≥ P + 1)

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

enum Phase { VALIDATE, NM_INIT, NM_ITER, NM_SHRINK, NM_FINAL, DONE };

struct Chain {
  std::vector<double> start;  // unconstrained start after sanitising and ×0.95 rescaling
  int n = 0;                // parameters (simplex dimension)
  Phase phase = VALIDATE;
  int window = 0;           // T_use of this chain
  std::vector<double> p;    // current unconstrained parameters
  int rescales = 0;
  double prev_ll = -INFINITY;
  int outer = 0;            // group iteration (1-based once the first Nelder–Mead starts)
  int status = YFM_OK;      // 0 ok, 1 the reference throws, 2 aborted after iteration 1
  // Nelder–Mead state (Optim's NelderMeadState)
  std::vector<double> S;    // (n+1) × n vertices, row v = vertex v
  std::vector<double> fs;   // n+1 vertex values
  std::vector<int> order;   // stable sortperm of fs
  int it = 0;
  bool converged = false;
  std::vector<double> xc, xl, trial;  // centroid, best vertex, requested points
  int n_req = 0;
  // speculation tree of this round (node 0 = the real iteration, see the file header)
  struct Node {
    int parent;  // -1 for node 0
    int src;     // the parent's accepted trial point: 0 reflection, 1 expansion, 2 outside, 3 inside
    int h;       // the worst vertex of this node's simplex
    int kind;    // outcome kind of the parent's iteration this node assumes (outcome_kind)
    int depth;   // iterations after the real one
    double prob; // estimated probability that the chain reaches this node
  };
  std::vector<Node> nodes;
  std::vector<const double*> vx;  // nodes × (n+1) vertex pointers (into S or an ancestor's points)
  std::vector<double> pts;        // nodes × 4n trial points (node 0's are also in trial)
  std::vector<double> xcs;        // centroid scratch
  std::vector<double> pre;        // (n+2) × n storage-order prefix sums of the simplex
  int acc_src = -1;               // accepted trial point of the last NM_ITER consume (-1: shrink)
  long long used = 0;             // evaluations consumed by the chain
  long long spec_hits = 0;
  long long depth_hist[8] = {};   // iterations consumed per round (stats)
  // outcome kind of each iteration (outcome_kind), previous → next; drives the tree's priorities
  int last_kind = 7;
  long long trans[8][8] = {};
  int last_h = -1;              // the vertex the previous iteration replaced
  long long recent[2] = {};     // "not the new vertex" outcomes: worst = last_h, all
};

// 0 reflection, 1 expansion, 2/3 outside contraction (3: the new vertex is the worst),
// 4/5 inside contraction (5: the new vertex is the worst), 6 shrink
int outcome_kind(const Chain& c, int ih) {
  if (c.acc_src < 0) return 6;
  const bool nw = c.order[c.n] == ih;
  return c.acc_src <= 1 ? c.acc_src : 2 * c.acc_src - 2 + (nw ? 1 : 0);
}

void sortperm(Chain& c) {
  std::iota(c.order.begin(), c.order.end(), 0);
  std::stable_sort(c.order.begin(), c.order.end(), [&](int a, int b) {
    const double fa = c.fs[a], fb = c.fs[b];
    if (std::isnan(fa) || std::isnan(fb)) return !std::isnan(fa) && std::isnan(fb);
    return fa < fb;
  });
}

// centroid of all vertices but h: storage-order sum × (1/n)   (Optim centroid!)
void centroid(const Chain& c, int h, double* out) {
  const int n = c.n;
  for (int k = 0; k < n; ++k) out[k] = 0.0;
  for (int v = 0; v <= n; ++v) {
    if (v == h) continue;
    const double* x = &c.S[(size_t)v * n];
    for (int k = 0; k < n; ++k) out[k] = out[k] + x[k];
  }
  const double r = 1.0 / n;
  for (int k = 0; k < n; ++k) out[k] = out[k] * r;
}

// sqrt(var(f) · n/(n+1)): population standard deviation of the vertex values
double nm_x(const Chain& c) {
  const int m = c.n + 1;
  double s = 0.0;
  for (int v = 0; v < m; ++v) s = s + c.fs[v];
  const double mu = s / m;
  double q = 0.0;
  for (int v = 0; v < m; ++v) {
    const double d = c.fs[v] - mu;
    q = q + d * d;
  }
  return std::sqrt(q / (m - 1) * ((double)(m - 1) / m));
}

struct Params {
  double al, be, ga, de;
};

Params nm_parameters(int n) {  // Optim.AdaptiveParameters: (α, β + 2/n, γ − 1/2n, δ − 1/n)
  return {1.0, 1.0 + 2.0 / n, 0.75 - 1.0 / (2.0 * n), 1.0 - 1.0 / n};
}

// Nelder–Mead trial points of the iteration whose worst vertex is h: centroid of the other
// vertices (storage order), then reflection, expansion, outside and inside contraction
// of the simplex whose vertex v is vx[v] (centroid! with the same operation order as centroid).
// pre = the storage-order partial sum of vertices 0..d−1 (0.0 + x_0 + … + x_{d−1}, as centroid
// forms it), valid when none of them is h or differs from the simplex pre was summed over.
void iter_trials(int n, const double* const* vx, int h, double* xc, double* trial, const double* pre, int d) {
  const Params q = nm_parameters(n);
  double acc[kMaxSlot];  // a local accumulator: no aliasing with the vertices, so it vectorises
  for (int k = 0; k < n; ++k) acc[k] = pre[k];
  for (int v = d; v <= n; ++v) {
    if (v == h) continue;
    const double* __restrict x = vx[v];
    for (int k = 0; k < n; ++k) acc[k] = acc[k] + x[k];
  }
  const double r = 1.0 / n;
  for (int k = 0; k < n; ++k) xc[k] = acc[k] * r;
  const double* xh = vx[h];
  double* xr = trial;
  for (int k = 0; k < n; ++k) xr[k] = xc[k] + q.al * (xc[k] - xh[k]);
  for (int k = 0; k < n; ++k) {
    const double d = xr[k] - xc[k];
    trial[n + k] = xc[k] + q.be * d;      // expansion
    trial[2 * n + k] = xc[k] + q.ga * d;  // outside contraction
    trial[3 * n + k] = xc[k] - q.ga * d;  // inside contraction
  }
}

// Speculation tree of an NM_ITER round (see the file header).  Node 0 is the real iteration on
// the chain's simplex.  A child of node X assumes one way X's iteration ends without a shrink:
// the accepted trial point src replaces X's worst vertex h_X, and hp is the worst vertex of the
// result — h_X itself (only after a contraction), the worst vertex whose value is already known,
// or one replaced earlier on the path (its value is not known yet).  Nodes are chosen best-first
// by the estimated probability that the chain reaches them (products of the chain's own
// outcome-transition frequencies), which maximises the expected iterations per round for the
// node budget.  Every node's trial points are computed exactly as the real iteration would
// compute them from that simplex (iter_trials on the same vertex coordinates, same worst index).
constexpr int kMaxNodes = 32;
constexpr int kMaxGroups = 4;

void build_tree(Chain& c, int budget, int max_depth) {
  const int n = c.n, m = n + 1;
  const size_t w = (size_t)4 * n;
  budget = std::max(1, std::min(budget, kMaxNodes));
  c.nodes.clear();
  c.nodes.reserve(budget);
  c.vx.resize((size_t)budget * m);
  c.pts.resize((size_t)budget * w);  // sized once: children point into it
  c.xcs.resize(n);
  // pre[v] = 0.0 + x_0 + … + x_{v−1} over the chain's simplex: every node's centroid sum starts
  // from the longest prefix of vertices it shares with it
  c.pre.resize((size_t)(m + 1) * n);
  for (int k = 0; k < n; ++k) c.pre[k] = 0.0;
  for (int v = 0; v < m; ++v)
    for (int k = 0; k < n; ++k) c.pre[(size_t)(v + 1) * n + k] = c.pre[(size_t)v * n + k] + c.S[(size_t)v * n + k];
  auto trials = [&](const double* const* v, int h, double* out) {
    int d = 0;
    while (d < h && v[d] == &c.S[(size_t)d * n]) ++d;
    iter_trials(n, v, h, c.xcs.data(), out, &c.pre[(size_t)d * n], d);
  };
  c.nodes.push_back({-1, -1, c.order[n], c.last_kind, 0, 1.0});
  for (int v = 0; v < m; ++v) c.vx[v] = &c.S[(size_t)v * n];
  trials(c.vx.data(), c.order[n], c.pts.data());
  if (budget == 1 || max_depth <= 0) return;
  // P(next kind | previous kind) from the chain's counts plus one pseudo-count per kind;
  // rq: share of "not the new vertex" outcomes whose worst is the previously replaced vertex
  double pk[8][7];
  bool pk_ok[8] = {};
  auto row_of = [&](int a) -> const double* {
    if (!pk_ok[a]) {
      double t = 0.0;
      for (int k = 0; k < 7; ++k) t += (double)c.trans[a][k] + 1.0;
      for (int k = 0; k < 7; ++k) pk[a][k] = ((double)c.trans[a][k] + 1.0) / t;
      pk_ok[a] = true;
    }
    return pk[a];
  };
  const double rq = ((double)c.recent[0] + 1.0) / ((double)c.recent[1] + 2.0);
  struct Cand {
    int parent, src, h, kind;
    double prob;
  };
  Cand cand[kMaxNodes * 4 * 8];  // a max-heap on prob
  int nc = 0;
  auto by_prob = [](const Cand& a, const Cand& b) { return a.prob < b.prob; };
  auto expand = [&](int x) {
    const Chain::Node X = c.nodes[x];
    if (X.depth >= max_depth) return;
    int uu[kMaxNodes];  // the vertices replaced on the path to X other than h_X (values unknown)
    int nu = 0;
    for (int p = x; c.nodes[p].parent >= 0; p = c.nodes[p].parent) {
      const int u = c.nodes[c.nodes[p].parent].h;
      bool seen = u == X.h;
      for (int q = 0; q < nu && !seen; ++q) seen = uu[q] == u;
      if (!seen) uu[nu++] = u;
    }
    int wk = -1;  // the worst vertex with a known value
    for (int i = n; i >= 0 && wk < 0; --i) {
      const int v = c.order[i];
      bool rep = v == X.h;
      for (int q = 0; q < nu && !rep; ++q) rep = uu[q] == v;
      if (!rep) wk = v;
    }
    const double* row = row_of(X.kind);
    auto push = [&](int src, int h, int kind, double p) {
      if (p < 5e-3 || nc >= (int)(sizeof(cand) / sizeof(cand[0]))) return;  // never among the top nodes
      cand[nc++] = {x, src, h, kind, p};
      std::push_heap(cand, cand + nc, by_prob);
    };
    for (int src = 0; src < 4; ++src) {
      const int kn = src <= 1 ? src : 2 * src - 2;  // the new vertex is not the worst
      if (src >= 2) push(src, X.h, kn + 1, X.prob * row[kn + 1]);
      const double pn = X.prob * row[kn];
      if (wk >= 0) push(src, wk, kn, pn * (nu ? 1.0 - rq : 1.0));
      for (int q = 0; q < nu; ++q) push(src, uu[q], kn, pn * rq / nu);
    }
  };
  expand(0);
  while ((int)c.nodes.size() < budget && nc > 0) {
    std::pop_heap(cand, cand + nc, by_prob);
    const Cand k = cand[--nc];
    const int id = (int)c.nodes.size();
    const Chain::Node P = c.nodes[k.parent];
    c.nodes.push_back({k.parent, k.src, k.h, k.kind, P.depth + 1, k.prob});
    const double** v = &c.vx[(size_t)id * m];
    std::copy(&c.vx[(size_t)k.parent * m], &c.vx[(size_t)(k.parent + 1) * m], v);
    v[P.h] = &c.pts[(size_t)k.parent * w + (size_t)k.src * n];
    trials(v, k.h, &c.pts[(size_t)id * w]);
    expand(id);
  }
}

// Queue the points chain c needs this round; advances phases that need no evaluation.
void prepare(Chain& c, int iterations, int spec_nodes) {
  const int n = c.n, m = n + 1;
  c.n_req = 0;
  c.nodes.clear();
  if (c.phase == NM_ITER && (c.converged || c.it >= iterations)) c.phase = NM_FINAL;
  c.trial.clear();
  switch (c.phase) {
    case VALIDATE:
      c.trial = c.p;
      break;
    case NM_INIT: {  // AffineSimplexer(a = 0.025, b = 0.5)
      c.S.assign((size_t)m * n, 0.0);
      for (int v = 0; v < m; ++v) std::copy(c.p.begin(), c.p.end(), c.S.begin() + (size_t)v * n);
      for (int j = 0; j < n; ++j) {
        double& x = c.S[(size_t)(j + 1) * n + j];
        x = (1.0 + 0.5) * x + 0.025;
      }
      c.fs.assign(m, 0.0);
      c.order.assign(m, 0);
      c.it = 0;
      c.converged = false;
      c.last_kind = 7;
      c.trial = c.S;
      break;
    }
    case NM_ITER:
      build_tree(c, spec_nodes, iterations - c.it - 1);
      c.trial.assign(c.pts.begin(), c.pts.begin() + (size_t)4 * n);
      break;
    case NM_SHRINK: {
      const Params q = nm_parameters(n);
      c.trial.assign((size_t)n * n, 0.0);
      for (int i = 1; i < m; ++i) {
        double* x = &c.S[(size_t)c.order[i] * n];
        for (int k = 0; k < n; ++k) x[k] = c.xl[k] + q.de * (x[k] - c.xl[k]);
        std::copy(x, x + n, c.trial.begin() + (size_t)(i - 1) * n);
      }
      break;
    }
    case NM_FINAL: {  // after_while!: centroid of all but the worst, after a final sortperm
      sortperm(c);
      c.xc.assign(n, 0.0);
      centroid(c, c.order[m - 1], c.xc.data());
      c.trial = c.xc;
      break;
    }
    case DONE:
      return;
  }
  c.n_req = (int)(c.trial.size() / n);
}

// Minimal fork-join pool for the per-round host work (chains are independent).
class Pool {
 public:
  explicit Pool(int n) {
    for (int i = 1; i < n; ++i) th_.emplace_back([this] { worker(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
      stop_a_.store(true, std::memory_order_release);
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // f(i) for i in [0, n), items handed out in chunks; returns when all are done
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
      ++gen_;
      gen_a_.store(gen_, std::memory_order_release);
      wake = sleepers_ > 0;
    }
    if (wake) cv_.notify_all();
    drain();
    while (done_.load(std::memory_order_acquire) < n) __builtin_ia32_pause();
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
      done_.fetch_add(i1 - i0, std::memory_order_release);
    }
  }
  // Rounds come every few hundred µs: a worker spins for the next one (a futex wake-up costs tens
  // of µs per thread) and only sleeps after 2 ms without work.
  void worker() {
    int seen = 0;
    for (;;) {
      const auto t0 = std::chrono::steady_clock::now();
      for (int k = 0; gen_a_.load(std::memory_order_acquire) == seen && !stop_a_.load(std::memory_order_acquire); ++k) {
        __builtin_ia32_pause();
        if ((k & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
      }
      {
        std::unique_lock<std::mutex> lk(m_);
        if (!stop_ && gen_ == seen) {
          ++sleepers_;
          cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
          --sleepers_;
        }
        if (stop_) return;
        if (!job_) {  // the round this generation announced is already over
          seen = gen_;
          continue;
        }
        seen = gen_;
      }
      drain();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_;
  std::function<void(int)>* job_ = nullptr;
  int n_ = 0, chunk_ = 1, gen_ = 0, sleepers_ = 0;
  bool stop_ = false;
  std::atomic<int> next_{0}, done_{0}, gen_a_{0};
  std::atomic<bool> stop_a_{false};
};

// objective values −loglik of this chain's requests; NaN ⇔ compute_loss threw
void fail(Chain& c) {
  // the optimizer threw: rethrown on the first group iteration (the estimation fails),
  // later the chain keeps its parameters and stops (optimization.jl:249-257)
  c.status = c.outer <= 1 ? 1 : 2;
  c.phase = DONE;
}

void consume(Chain& c, const double* f, int max_group_iters, double tol, double g_tol) {
  const int n = c.n, m = n + 1;
  switch (c.phase) {
    case VALIDATE: {
      if (std::isnan(f[0])) {
        c.status = 1;
        c.phase = DONE;
        return;
      }
      const double ll = -f[0];
      if (!std::isfinite(ll) && c.rescales < 10) {
        for (double& x : c.p) x = x * 0.95;
        ++c.rescales;
        return;
      }
      c.outer = 1;
      c.start = c.p;  // the sanitised, rescaled start: estimate_steps!'s init_p (optimization.jl:281, :298-302)
      c.phase = NM_INIT;
      return;
    }
    case NM_INIT:
      for (int v = 0; v < m; ++v) {
        if (std::isnan(f[v])) return fail(c);
        c.fs[v] = f[v];
      }
      sortperm(c);
      c.phase = NM_ITER;
      return;
    case NM_ITER: {
      ++c.it;
      c.acc_src = -1;
      const int il = c.order[0], ish = c.order[n - 1], ih = c.order[m - 1];
      const double fl = c.fs[il], fsh = c.fs[ish], fh = c.fs[ih];
      c.xl.assign(c.S.begin() + (size_t)il * n, c.S.begin() + (size_t)(il + 1) * n);
      const double fr = f[0];
      if (std::isnan(fr)) return fail(c);
      double* xh = &c.S[(size_t)ih * n];
      const double* xr = &c.trial[0];
      bool shrink = false;
      if (fr < fl) {
        const double fe = f[1];
        if (std::isnan(fe)) return fail(c);
        if (fe < fr) {
          std::copy(&c.trial[n], &c.trial[2 * n], xh);
          c.fs[ih] = fe;
          c.acc_src = 1;
        } else {
          std::copy(xr, xr + n, xh);
          c.fs[ih] = fr;
          c.acc_src = 0;
        }
        for (int i = m - 1; i >= 1; --i) c.order[i] = c.order[i - 1];  // the new vertex is the lowest
        c.order[0] = ih;
      } else if (fr < fsh) {
        std::copy(xr, xr + n, xh);
        c.fs[ih] = fr;
        c.acc_src = 0;
        sortperm(c);
      } else if (fr < fh) {
        const double fo = f[2];
        if (std::isnan(fo)) return fail(c);
        if (fo < fr) {
          std::copy(&c.trial[2 * n], &c.trial[3 * n], xh);
          c.fs[ih] = fo;
          c.acc_src = 2;
          sortperm(c);
        } else {
          shrink = true;
        }
      } else {
        const double fi = f[3];
        if (std::isnan(fi)) return fail(c);
        if (fi < fh) {
          std::copy(&c.trial[3 * n], &c.trial[4 * n], xh);
          c.fs[ih] = fi;
          c.acc_src = 3;
          sortperm(c);
        } else {
          shrink = true;
        }
      }
      if (shrink) {
        c.phase = NM_SHRINK;
        return;
      }
      c.converged = nm_x(c) <= g_tol;
      return;
    }
    case NM_SHRINK:
      for (int i = 1; i < m; ++i) {
        if (std::isnan(f[i - 1])) return fail(c);
        c.fs[c.order[i]] = f[i - 1];
      }
      sortperm(c);
      c.converged = nm_x(c) <= g_tol;
      c.phase = NM_ITER;
      return;
    case NM_FINAL: {
      const double fcm = f[0];
      if (std::isnan(fcm)) return fail(c);
      int imin = 0;
      for (int v = 1; v < m; ++v)
        if (c.fs[v] < c.fs[imin]) imin = v;  // findmin: first minimum
      double fmin = c.fs[imin];
      const double* xmin = &c.S[(size_t)imin * n];
      if (fcm < fmin) {
        xmin = c.xc.data();
        fmin = fcm;
      }
      c.p.assign(xmin, xmin + n);
      // ll = −loss_wrapper(p) (:269): the objective at the minimizer, already evaluated
      const double ll = -fmin;
      const double d = ll - c.prev_ll;
      if (std::fabs(d) < tol) {
        c.prev_ll = ll;
        c.phase = DONE;
        return;
      }
      c.prev_ll = ll;
      if (c.outer >= max_group_iters) {
        c.phase = DONE;
        return;
      }
      ++c.outer;
      c.phase = NM_INIT;
      return;
    }
    case DONE:
      return;
  }
}

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
      // outcome statistics of every NM iteration: they set the speculation tree's priorities
      auto note = [&](int ih) {
        if (c.phase == DONE) return;
        const int k = outcome_kind(c, ih);
        ++c.trans[c.last_kind][k];
        c.last_kind = k;
        if (k == 0 || k == 1 || k == 2 || k == 4) {
          ++c.recent[1];
          if (c.order[c.n] == c.last_h && c.last_h != ih) ++c.recent[0];
        }
        c.last_h = ih;
      };
      const Phase ph0 = c.phase;
      const int ih0 = ph0 == NM_ITER ? c.order[c.n] : -1;
      consume(c, f, max_group_iters, tol, g_tol);
      c.used += c.n_req;
      if (ph0 == NM_ITER) {
        note(ih0);
        // walk down the speculation tree while the chain's real state is a speculated node's
        int cur = 0, done = 1;
        const size_t w = (size_t)4 * c.n;
        while (c.phase == NM_ITER && c.acc_src >= 0 && !c.converged && c.it < iterations) {
          const int hp = c.order[c.n];
          int nxt = -1;
          for (int k = 1; k < (int)c.nodes.size(); ++k)
            if (c.nodes[k].parent == cur && c.nodes[k].src == c.acc_src && c.nodes[k].h == hp) {
              nxt = k;
              break;
            }
          if (nxt < 0) break;
          c.trial.assign(c.pts.begin() + nxt * w, c.pts.begin() + (nxt + 1) * w);
          consume(c, f + 4 * nxt, max_group_iters, tol, g_tol);
          note(hp);
          c.used += 4;
          ++c.spec_hits;
          cur = nxt;
          ++done;
        }
        ++c.depth_hist[std::min(done, 7)];
      }
      c.nodes.clear();
    }
    const auto h1 = stats ? clk::now() : clk::time_point();
    prepare(c, iterations, spec_nodes);
    const auto h2 = stats ? clk::now() : clk::time_point();
    if (c.n_req > 0) {
      active.fetch_add(1, std::memory_order_relaxed);
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
  auto host_group = [&](int g) {
    active.store(0);
    pool.run(r0[g + 1] - r0[g], 2, [&](int i) { host_step(r0[g] + i); });
    return active.load() > 0;
  };
  auto submit = [&](int g) -> int {
    const size_t o = (size_t)r0[g] * SLOT;
    const int Bg = (r0[g + 1] - r0[g]) * SLOT;
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

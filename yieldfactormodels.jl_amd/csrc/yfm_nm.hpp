// yfm_nm.hpp — the host side of the batched estimation driver (yfm_estimate.hip) that needs no
// device: one estimate_steps! chain as a state machine (Optim.jl NelderMead restated), the
// speculation tree of later iterations, and absorb(), which consumes one round's objective values
// (the real iteration, then the speculated iterations whose simplex the chain reaches).  Plain
// C++ so the CPU tests can drive it with a host objective (tests/test_nm_tree_cpu.py).
//
// Reference: src/optimization.jl:137-312 (estimate_steps!), :442-451, :479 (NelderMead opt1);
// Optim.jl 1.13 NelderMead (not vendored; restated, see yfm_estimate.hip's header).
#pragma once
#pragma clang fp contract(off)

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <vector>

#include "../../include/yfm.h"

namespace yfm_nm {

constexpr int kMaxSlot = 128;  // points per chain and round (≥ P + 1)

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
inline int outcome_kind(const Chain& c, int ih) {
  if (c.acc_src < 0) return 6;
  const bool nw = c.order[c.n] == ih;
  return c.acc_src <= 1 ? c.acc_src : 2 * c.acc_src - 2 + (nw ? 1 : 0);
}

inline void sortperm(Chain& c) {
  std::iota(c.order.begin(), c.order.end(), 0);
  std::stable_sort(c.order.begin(), c.order.end(), [&](int a, int b) {
    const double fa = c.fs[a], fb = c.fs[b];
    if (std::isnan(fa) || std::isnan(fb)) return !std::isnan(fa) && std::isnan(fb);
    return fa < fb;
  });
}

// centroid of all vertices but h: storage-order sum × (1/n)   (Optim centroid!)
inline void centroid(const Chain& c, int h, double* out) {
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
inline double nm_x(const Chain& c) {
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

inline Params nm_parameters(int n) {  // Optim.AdaptiveParameters: (α, β + 2/n, γ − 1/2n, δ − 1/n)
  return {1.0, 1.0 + 2.0 / n, 0.75 - 1.0 / (2.0 * n), 1.0 - 1.0 / n};
}

// Nelder–Mead trial points of the iteration whose worst vertex is h: centroid of the other
// vertices (storage order), then reflection, expansion, outside and inside contraction
// of the simplex whose vertex v is vx[v] (centroid! with the same operation order as centroid).
// pre = the storage-order partial sum of vertices 0..d−1 (0.0 + x_0 + … + x_{d−1}, as centroid
// forms it), valid when none of them is h or differs from the simplex pre was summed over.
inline void iter_trials(int n, const double* const* vx, int h, double* xc, double* trial, const double* pre, int d) {
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

inline void build_tree(Chain& c, int budget, int max_depth) {
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
inline void prepare(Chain& c, int iterations, int spec_nodes) {
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

// objective values −loglik of this chain's requests; NaN ⇔ compute_loss threw
inline void fail(Chain& c) {
  // the optimizer threw: rethrown on the first group iteration (the estimation fails),
  // later the chain keeps its parameters and stops (optimization.jl:249-257)
  c.status = c.outer <= 1 ? 1 : 2;
  c.phase = DONE;
}

inline void consume(Chain& c, const double* f, int max_group_iters, double tol, double g_tol) {
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


// One round's objective values f (the chain's slot: node k's four points at 4k, or the n_req
// points of a non-iteration phase) → the chain's state after the real iteration and every
// speculated one it reaches.  Returns the iterations consumed (0 outside NM_ITER).
inline int absorb(Chain& c, const double* f, int iterations, int max_group_iters, double tol, double g_tol) {
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
  int done = 0;
  if (ph0 == NM_ITER) {
    note(ih0);
    done = 1;
    // walk down the speculation tree while the chain's real state is a speculated node's
    int cur = 0;
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
  return done;
}

}  // namespace yfm_nm

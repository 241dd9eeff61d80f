// CPU driver of the estimation driver's host logic (yieldfactormodels.jl_amd/csrc/yfm_nm.hpp):
// R estimate_steps! chains on a host objective, rounds exactly as yfm_estimate runs them (prepare →
// evaluate the chain's slot → absorb), with a given speculation-tree budget.  Used by
// tests/test_nm_tree_cpu.py, which compares budgets with each other and with oracle/optim_nm.py.
//   nm_tree_check R n budget iterations max_group_iters
#include <cstdio>
#include <cstdlib>

#include "../yieldfactormodels.jl_amd/csrc/yfm_nm.hpp"

using namespace yfm_nm;

// deterministic, non-separable, evaluated left to right (the Python twin in the test does the same);
// +Inf where x₀ > 5 so that a start there goes through estimate_steps!'s ×0.95 rescaling
static double objective(const double* x, int n, int r) {
  if (x[0] > 5.0) return INFINITY;
  double s = 0.0;
  for (int i = 0; i < n; ++i) {
    const double d = x[i] - 0.1 * (i % 5) - 0.01 * r;
    s = s + (1.0 + 0.25 * (i % 3)) * d * d;
  }
  for (int i = 0; i + 1 < n; ++i) s = s + 0.05 * x[i] * x[i + 1];
  return s;
}

int main(int argc, char** argv) {
  if (argc < 6) return 2;
  const int R = std::atoi(argv[1]), n = std::atoi(argv[2]), budget = std::atoi(argv[3]);
  const int iterations = std::atoi(argv[4]), mgi = std::atoi(argv[5]);
  std::vector<Chain> ch(R);
  for (int r = 0; r < R; ++r) {
    Chain& c = ch[r];
    c.n = n;
    c.p.resize(n);
    for (int i = 0; i < n; ++i) c.p[i] = (0.2 * ((i * 7 + r * 3) % 11)) / 11.0 - 0.1;
    if (r == 0) c.p[0] = 6.0;
  }
  std::vector<double> fv(kMaxSlot);
  long long rounds = 0;
  for (bool any = true; any; ++rounds) {
    any = false;
    for (int r = 0; r < R; ++r) {
      Chain& c = ch[r];
      prepare(c, iterations, budget);
      if (c.n_req == 0) continue;
      any = true;
      const int npts = c.nodes.empty() ? c.n_req : 4 * (int)c.nodes.size();
      const double* pts = c.nodes.empty() ? c.trial.data() : c.pts.data();
      for (int k = 0; k < npts; ++k) fv[k] = objective(pts + (size_t)k * n, n, r);
      absorb(c, fv.data(), iterations, mgi, 1e-8, 1e-6);
    }
  }
  std::printf("rounds %lld\n", rounds);
  for (const Chain& c : ch) {
    std::printf("chain %d %lld %a", c.status, c.used, c.prev_ll);
    for (double x : c.p) std::printf(" %a", x);
    std::printf("\n");
  }
  return 0;
}

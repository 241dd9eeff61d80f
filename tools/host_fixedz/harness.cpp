// Host harness for the per-lane fixed-loading filter (csrc/yfm_fixedz.hpp): runs the GNS5 (M = 5) or DNS
// (M = 3) filter of the VALU-Z'ỹ kernel path (yfm_kernels.hip, NP > 32: no MFMA) one candidate at a time on
// the CPU, in the one-body form (collapsed_update) and the two-function form (collapsed_cov +
// collapsed_mean), and prints both logliks.  Built with clang++ -fsanitize=memory it checks the filter's
// C++ for reads of uninitialised values (tools/host_fixedz/run.sh).  Diagnostic only: not the product, not
// a parity reference (host exp/log/rcp differ from the device's).
//
//   harness <case.bin>      case.bin: int32 [N, T, B, P, space, has_tuse, kind], then f64 mats[N],
//                           Y[N·T] (column-major), Θ[P·B] (column-major), then int32 T_use[B] if has_tuse
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "yfm_fixedz.hpp"

using namespace yfm;

// z̃ = Z'ỹ_t as yfm_kernels.hip's dot_zt (two partial sums per column, the same order)
template <int NP, int NZ>
static void dot_zt(const double* col, const double (&Zc)[NZ][NP], double (&zt)[NZ]) {
  double a[NZ][2];
  for (int cz = 0; cz < NZ; ++cz) a[cz][0] = a[cz][1] = 0.0;
  for (int i = 0; i < NP; i += 2)
    for (int cz = 0; cz < NZ; ++cz) {
      a[cz][0] = fma(Zc[cz][i], col[i], a[cz][0]);
      a[cz][1] = fma(Zc[cz][i + 1], col[i + 1], a[cz][1]);
    }
  for (int cz = 0; cz < NZ; ++cz) zt[cz] = a[cz][0] + a[cz][1];
}

template <int NP, int M, int LEAD, bool SPLIT>
static std::vector<double> run(int N, int T, int B, int P, int space, const double* mats, const double* Y,
                               const double* Th, const int* T_use) {
  constexpr int LDP = NP + 4;
  constexpr int NZ = M - 1;
  // prep_panel_kernel: centered columns, ȳ, ỹ'ỹ, NaN flag, y'y
  std::vector<double> panel((size_t)T * LDP);
  for (int t = 0; t < T; ++t) {
    const double* y = Y + (size_t)t * N;
    double* o = panel.data() + (size_t)t * LDP;
    double s1 = 0.0, yy = 0.0;
    bool nan = false;
    for (int i = 0; i < N; ++i) {
      nan = nan || (y[i] != y[i]);
      s1 += y[i];
      yy = fma(y[i], y[i], yy);
    }
    const double ybar = s1 / (double)N;
    double tt = 0.0;
    for (int i = 0; i < N; ++i) {
      o[i] = y[i] - ybar;
      tt = fma(o[i], o[i], tt);
    }
    for (int i = N; i < NP; ++i) o[i] = 0.0;
    o[NP] = ybar;
    o[NP + 1] = tt;
    o[NP + 2] = nan ? 1.0 : 0.0;
    o[NP + 3] = yy;
  }
  std::vector<double> out(B, 0.0);
  unsigned flags[8] = {0};
  const int nwave = (B + 63) / 64;
  for (int w = 0; w < nwave; ++w) {
    // the wave's lanes: live lanes b < B; lanes past B mirror candidate B − 1 and are not live
    int wave_min_data = 0x7fffffff, nsteps = 0;
    for (int l = 0; l < 64; ++l) {
      const int b = w * 64 + l;
      if (b >= B) continue;
      const int nobs = T_use ? T_use[b] : T;
      wave_min_data = std::min(wave_min_data, nobs - 1);
    }
    // nsteps: the block's longest window (kBlock = 256 lanes = 4 waves)
    const int blk = w / 4;
    for (int b = blk * 256; b < std::min(B, blk * 256 + 256); ++b) nsteps = std::max(nsteps, (T_use ? T_use[b] : T) - 1);
    for (int l = 0; l < 64; ++l) {
      const int b = w * 64 + l;
      if (b >= B) break;
      const int nobs = T_use ? T_use[b] : T;
      const int my_steps = nobs - 1, my_data = nobs - 1;
      Params<M, LEAD> p;
      decode_params<M, LEAD>(Th + (size_t)b * P, space, p);
      double Zc[NZ][NP];
      for (int lg = 0; lg < LEAD; ++lg) {
        const double lam = 1e-2 + exp(p.gam[lg]);
        for (int i = 0; i < NP; ++i) {
          if (i < N) {
            const double tau = lam * mats[i];
            const double z = exp(-tau);
            const double s = (1.0 - z) / tau;
            Zc[2 * lg][i] = s;
            Zc[2 * lg + 1][i] = s - z;
          } else {
            Zc[2 * lg][i] = 0.0;
            Zc[2 * lg + 1][i] = 0.0;
          }
        }
      }
      double G[M][M];
      G[0][0] = (double)N;
      for (int c = 0; c < NZ; ++c) {
        double s = 0.0;
        for (int i = 0; i < NP; ++i) s += Zc[c][i];
        G[0][c + 1] = s;
        G[c + 1][0] = s;
        for (int d = c; d < NZ; ++d) {
          double g = 0.0;
          for (int i = 0; i < NP; ++i) g = fma(Zc[c][i], Zc[d][i], g);
          G[c + 1][d + 1] = g;
          G[d + 1][c + 1] = g;
        }
      }
      FixedZFilter<M, LEAD, false, false, SPLIT> f;
      f.p = p;
      f.steady_ok = false;
      f.setup(G, N, true);
      if (!f.collapsed) {  // deferred to the double-double kernel on the GPU
        out[b] = NAN;
        continue;
      }
      for (int t = 0; t < nsteps; ++t) {
        const double* c = panel.data() + (size_t)t * LDP;
        double zc[NZ];
        dot_zt<NP, NZ>(c, Zc, zc);
        const double2 yb = {c[NP], c[NP + 1]};
        const double2 meta = {c[NP + 2], c[NP + 3]};
        const bool fast = (t >= 1) && (meta.x == 0.0) && (t < wave_min_data);
        f.step(t, zc, yb, meta, fast, my_steps, my_data);
      }
      out[b] = f.loglik(nobs, flags);
    }
  }
  return out;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* fp = std::fopen(argv[1], "rb");
  if (!fp) return 2;
  int32_t h[7];
  if (std::fread(h, sizeof(int32_t), 7, fp) != 7) return 2;
  const int N = h[0], T = h[1], B = h[2], P = h[3], space = h[4], has_tuse = h[5], kind = h[6];
  std::vector<double> mats(N), Y((size_t)N * T), Th((size_t)P * B);
  std::vector<int> tu(B);
  if (std::fread(mats.data(), 8, N, fp) != (size_t)N || std::fread(Y.data(), 8, Y.size(), fp) != Y.size() ||
      std::fread(Th.data(), 8, Th.size(), fp) != Th.size())
    return 2;
  if (has_tuse && std::fread(tu.data(), 4, B, fp) != (size_t)B) return 2;
  std::fclose(fp);
  const int* T_use = has_tuse ? tu.data() : nullptr;
  std::vector<double> one, two;
  if (kind == 2) {  // GNS5, NP = 48 (N in 33..48)
    one = run<48, 5, 2, false>(N, T, B, P, space, mats.data(), Y.data(), Th.data(), T_use);
    two = run<48, 5, 2, true>(N, T, B, P, space, mats.data(), Y.data(), Th.data(), T_use);
  } else {  // DNS, NP = 48
    one = run<48, 3, 1, false>(N, T, B, P, space, mats.data(), Y.data(), Th.data(), T_use);
    two = run<48, 3, 1, true>(N, T, B, P, space, mats.data(), Y.data(), Th.data(), T_use);
  }
  int differ = 0;
  for (int b = 0; b < B; ++b) {
    const bool same = (one[b] == two[b]) || (one[b] != one[b] && two[b] != two[b]);
    differ += !same;
    std::printf("b %2d one % .17e two % .17e%s\n", b, one[b], two[b], same ? "" : "  <-- differ");
  }
  std::printf("differing: %d\n", differ);
  return 0;
}

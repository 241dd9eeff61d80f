// Reduced reproducer of the ROCm 7.2 AMDGPU VGPR→AGPR spill miscompile fenced by
// `-mllvm -amdgpu-spill-vgpr-to-agpr=0` in yieldfactormodels.jl_amd/build_native.py.
//
// One case (case2431.bin: GNS5, N = 33 → the NP = 48 per-lane kernel fixedz_loglik_kernel<48,5,2,…>, which
// spills ≈1.8 KB of VGPRs per lane, T = 3: one prediction step then one data step, 24 candidates), run
// through the C ABI (include/yfm.h) of a given libyfm_hip.so in both forms of the measurement update: the
// one-body collapsed_update and the two-function collapsed_cov + collapsed_mean (YFM_FZ_SPLIT_FORM=1, a
// diagnostic instantiation).  Both forms are the same arithmetic (explicit fma, FP contraction off), so a
// correct build gives bitwise equal logliks.  Exit status: 0 when they are equal, 1 when they differ.
//
//   ./repro <libyfm_hip.so> <case2431.bin>
#include <dlfcn.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef void* (*create_t)(int);
typedef void (*destroy_t)(void*);
typedef int (*set_panel_t)(void*, const double*, int, int, const double*);
typedef int (*loglik_t)(void*, int, int, const double*, int, int, const int*, double*);
typedef const char* (*err_t)(void);

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <libyfm_hip.so> <case.bin>\n", argv[0]);
    return 2;
  }
  void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    std::fprintf(stderr, "dlopen: %s\n", dlerror());
    return 2;
  }
  auto create = (create_t)dlsym(h, "yfm_create");
  auto destroy = (destroy_t)dlsym(h, "yfm_destroy");
  auto set_panel = (set_panel_t)dlsym(h, "yfm_set_panel");
  auto loglik = (loglik_t)dlsym(h, "yfm_loglik_batch");
  auto last_error = (err_t)dlsym(h, "yfm_last_error");
  FILE* f = std::fopen(argv[2], "rb");
  if (!f) return 2;
  int hdr[7];
  if (std::fread(hdr, sizeof(int), 7, f) != 7) return 2;
  const int kind = hdr[0], N = hdr[1], T = hdr[2], P = hdr[3], B = hdr[4], space = hdr[5], has_tu = hdr[6];
  std::vector<double> mats(N), Y((size_t)N * T), th((size_t)P * B);
  std::vector<int> tu(B);
  bool ok = std::fread(mats.data(), 8, N, f) == (size_t)N && std::fread(Y.data(), 8, Y.size(), f) == Y.size() &&
            std::fread(th.data(), 8, th.size(), f) == th.size() &&
            (!has_tu || std::fread(tu.data(), 4, B, f) == (size_t)B);
  std::fclose(f);
  if (!ok) return 2;
  void* ctx = create(0);
  if (!ctx || set_panel(ctx, Y.data(), N, T, mats.data()) != 0) {
    std::fprintf(stderr, "setup: %s\n", last_error());
    return 2;
  }
  std::vector<double> one(B), two(B);
  setenv("YFM_DNS_STEADY", "0", 1);  // the diagnostic instantiations are the full recursion
  unsetenv("YFM_FZ_SPLIT_FORM");
  int rc1 = loglik(ctx, kind, space, th.data(), P, B, has_tu ? tu.data() : nullptr, one.data());
  setenv("YFM_FZ_SPLIT_FORM", "1", 1);
  int rc2 = loglik(ctx, kind, space, th.data(), P, B, has_tu ? tu.data() : nullptr, two.data());
  if (rc1 || rc2) {
    std::fprintf(stderr, "loglik: %s\n", last_error());
    return 2;
  }
  int differ = 0;
  for (int b = 0; b < B; ++b) {
    const bool same = std::memcmp(&one[b], &two[b], 8) == 0 || (std::isnan(one[b]) && std::isnan(two[b]));
    differ += !same;
    std::printf("b %2d  one-body % .17g  two-function % .17g%s\n", b, one[b], two[b], same ? "" : "   DIFFER");
  }
  std::printf("%s: %d of %d candidates differ between the two forms\n", argv[1], differ, B);
  destroy(ctx);
  return differ ? 1 : 0;
}

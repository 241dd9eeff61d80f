// dd_exp_check.hip — host-side accuracy check of the certified kernels' dd_exp (yfm_dd.hpp: dd_exp_core, the table
// version) and of the Taylor-and-squarings version it replaced, against binary128 expq on 10⁶ arguments.
//   hipcc -O2 --offload-arch=gfx950 -I yieldfactormodels.jl_amd/csrc tools/dd_exp_check.hip -lquadmath -o tools/dd_exp_check
// Prints the largest and the 99.9th-percentile relative error in units of u² = 2^-106 per argument range.
#include <quadmath.h>

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "yfm_dd.hpp"

using yfm::dd;

static const double kTab[128][2] = {
#include "yfm_exp_table.inc"
};

// the round-5 dd_exp: k·ln2 reduction, degree-9 Taylor on r/2^9, nine squarings of (1 + s)
static dd exp_old(dd x) {
  using namespace yfm;
  constexpr double kLn2Hi = 0.6931471805599453094172321214581766;
  constexpr double kLn2Lo = 2.3190468138462996154e-17;
  if (!(x.hi > -745.2)) return {x.hi != x.hi ? x.hi : 0.0, 0.0};
  if (x.hi > 709.8) return {__builtin_inf(), 0.0};
  const double k = __builtin_rint(x.hi * 1.4426950408889634073599);
  const dd kh = two_prod(k, kLn2Hi);
  dd r = dd_sub(x, kh);
  r = dd_add_d(r, -k * kLn2Lo);
  r = dd_ldexp(r, -9);
  const double f[10] = {1.0, 1.0, 0.5, 1.6666666666666666574e-01, 4.1666666666666664354e-02, 8.3333333333333332177e-03,
                        1.3888888888888889419e-03, 1.9841269841269841253e-04, 2.4801587301587301566e-05,
                        2.7557319223985892511e-06};
  const double fl[10] = {0.0, 0.0, 0.0, 9.2518585385429706566e-18, 2.3129646346357426641e-18, 1.1564823173178713802e-19,
                         -5.3005439543735770590e-20, 1.7209558293420705286e-22, 2.1511947866775881608e-23,
                         -1.8583932740464720810e-22};
  dd p = {f[9], fl[9]};
  for (int n = 8; n >= 1; --n) p = dd_add(dd_mul(p, r), dd{f[n], fl[n]});
  dd s = dd_mul(p, r);
  for (int i = 0; i < 9; ++i) s = dd_mul(s, dd_add_d(s, 2.0));
  return dd_ldexp(dd_add_d(s, 1.0), (int)k);
}

static double rel_u2(dd got, __float128 ref) {
  const __float128 g = (__float128)got.hi + (__float128)got.lo;
  if (ref == 0) return g == 0 ? 0.0 : 1e300;
  __float128 e = (g - ref) / ref;
  if (e < 0) e = -e;
  return (double)(e * (__float128)0x1p106);
}

int main() {
  std::mt19937_64 rng(20261018);
  const double ranges[][2] = {{-1e-3, 1e-3}, {-1.0, 1.0}, {-40.0, 5.0}, {-400.0, 0.0}, {-600.0, 700.0}};  // below e^−672 the lo part is subnormal (both versions alike)
  int bad = 0;
  for (const auto& rg : ranges) {
    std::uniform_real_distribution<double> U(rg[0], rg[1]), V(-1.0, 1.0);
    std::vector<double> en, eo;
    const int n = 200000;
    for (int i = 0; i < n; ++i) {
      const double hi = U(rng);
      dd x = yfm::two_sum(hi, V(rng) * 1e-17 * (hi == 0 ? 1.0 : __builtin_fabs(hi)));
      const __float128 ref = expq((__float128)x.hi + (__float128)x.lo);
      en.push_back(rel_u2(yfm::dd_exp_core(x, kTab), ref));
      eo.push_back(rel_u2(exp_old(x), ref));
    }
    std::sort(en.begin(), en.end());
    std::sort(eo.begin(), eo.end());
    const double mn = en.back(), mo = eo.back();
    std::printf("x in [%g, %g]: table max %.2f u² (p99.9 %.2f), old max %.2f u² (p99.9 %.2f)\n", rg[0], rg[1], mn,
                en[(size_t)(0.999 * n)], mo, eo[(size_t)(0.999 * n)]);
    if (mn > 2.0 * mo + 8.0) ++bad;
  }
  std::printf(bad ? "FAIL\n" : "ok\n");
  return bad;
}

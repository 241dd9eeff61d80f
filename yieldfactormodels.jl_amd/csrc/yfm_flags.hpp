// yfm_flags.hpp — layout of the per-launch device counters (shared by the kernels and the C ABI).
#pragma once

namespace yfm {

// two banks of kFlagsPerBank unsigned ints: [0] n_init_throw, [1] n_neg_inf, [2] deferral list length,
// [3] n_deferred, [4] steady wave-steps of the DNS kernel (yfm_last_batch_steady), [5..7] spare.  A launch
// uses the bank its predecessor zeroed; its first kernel zeroes the other one.
constexpr int kFlagsPerBank = 8;

}  // namespace yfm

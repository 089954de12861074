// vx_sort.hpp — the rocprim radix-sort configuration of the device plan / map builds.
#pragma once
#include <rocprim/rocprim.hpp>

namespace vx {
// Stable LSD radix sort of (key, value) pairs over the low key bits.  rocprim's default picks its
// merge sort up to 2^20 items (a block sort, then ~log2(n / 1024) merge passes of two launches each);
// the builds here sort keys of few bits (6-17: keyframe rows, landmark slots, block indices), where
// the onesweep form needs one histogram launch and one launch per 8-bit digit, so the merge limit
// is 0.  Both forms are stable, so the sorted output is the same.
using OnesweepSort = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                rocprim::default_config, 0>;
}  // namespace vx

// Weight prefetch sweep (csrc/hip/prefetch.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mio {

// Reads [p, p + bytes) on n_wg 256-thread workgroups, discarding the data.
void launch_touch(const void *p, uint64_t bytes, int n_wg, hipStream_t s);

}  // namespace mio

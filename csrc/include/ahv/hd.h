// Common attributes for code that is compiled once and instantiated for both
// the host (scalar API path, CPU-side equivalence tests) and gfx950 (batched
// kernels).  Every translation unit in csrc/ is compiled by hipcc with
// --offload-arch=gfx950, so __host__/__device__ are always defined.
#pragma once

#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

#define AHV_HD __host__ __device__ __forceinline__

namespace ahv {

// Device-side sentinel for "no value" in int32 id columns.
constexpr int32_t kNone = -1;

// Batch counters are accumulated into kStatSpread rows (row = workgroup mod
// kStatSpread) and summed by the launcher afterwards: tens of thousands of waves
// adding to one address serialise at L2 (measured 0.5 ms for 16k waves × 4
// counters on MI355X); spread over 64 rows the contention disappears.
constexpr int kStatSpread = 64;

}  // namespace ahv

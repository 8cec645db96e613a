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

}  // namespace ahv

// Host-side declarations of kernel launchers and their CPU twins.
#pragma once

#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "ahv/hd.h"

namespace ahv {

inline void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// Fold [kStatSpread, k] spread counters into out[k] and re-zero them (one wave).
void launch_spread_fold(unsigned long long* spread, unsigned long long* out, int k, bool accumulate, hipStream_t s);

// Device time base and cursor maintenance for graph-captured pipelines (N07/N09).
// cursor = int64[3] {slot_base, id_base, now_us}.
void launch_pipeline_clock(int64_t* cursor, int64_t base_us, int64_t base_clk, int64_t rate_khz, hipStream_t s);
void launch_pipeline_advance(int64_t* cursor, int64_t n, int64_t capacity, hipStream_t s);
void launch_pipeline_epilogue(unsigned long long* spread, unsigned long long* out, int k, int64_t* cursor, int64_t n,
                              int64_t capacity, int64_t base_us, int64_t base_clk, int64_t rate_khz, hipStream_t s);
int64_t device_wall_clock(int device);  // one synchronous sample of wall_clock64()
int64_t device_wall_clock_rate_khz(int device);

// Kernel registry for resource introspection (hipFuncGetAttributes): every
// kernel translation unit lists its hot kernels; tests assert no scratch spills
// and the designed LDS footprint (agent_hypervisor_amd._C.kernel_attributes).
struct KernelEntry {
  const char* name;
  const void* fn;
};
void kernels_audit(std::vector<KernelEntry>& out);
void kernels_liability(std::vector<KernelEntry>& out);
void kernels_saga(std::vector<KernelEntry>& out);
void kernels_merkle_tree(std::vector<KernelEntry>& out);
void kernels_store_template(std::vector<KernelEntry>& out);

}  // namespace ahv

// Support kernels of the batched pipeline (csrc/hip/store_template.hip): the
// device time base and cursor of hipGraph-captured steps (N07/N09) and the fold
// of spread batch counters (X04 input).
#include <cstdlib>

#include "ahv/launch.h"
#include "ahv/pipeline.h"
#include "ahv/wave_sink.h"

namespace ahv {

// ---------------------------------------------------------- cursor kernels
// wall_clock64() is the constant-rate counter (hipDeviceAttributeWallClockRate);
// the host pairs one sample with its own UTC clock once, after which captured
// graphs stamp every replay with device-side "now" and no host round trip.

__global__ void pipeline_clock_kernel(int64_t* cursor, int64_t base_us, int64_t base_clk, int64_t rate_khz) {
  const int64_t ticks = static_cast<int64_t>(wall_clock64()) - base_clk;
  cursor[2] = base_us + ticks * 1000 / rate_khz;
}

__global__ void pipeline_advance_kernel(int64_t* cursor, int64_t n, int64_t capacity) {
  cursor[0] = (cursor[0] + n) % capacity;
  cursor[1] += 3 * n;
}

__global__ void wall_clock_kernel(int64_t* out) { *out = static_cast<int64_t>(wall_clock64()); }

// Spread-counter fold: one wave, lane = spread row.  Each row is read and zeroed
// in place (the next launch starts from zero without a fill), summed across the
// wave and added (or copied) into out[k].  One launch instead of zero + reduce + add.
constexpr int kMaxFold = 8;

__global__ __launch_bounds__(kWaveLanes) void spread_fold_kernel(unsigned long long* spread, unsigned long long* out,
                                                                 int k, int accumulate) {
  static_assert(kStatSpread == kWaveLanes, "one spread row per lane");
  const int lane = threadIdx.x;
  // all loads issued before the first use: one memory latency, not k
  unsigned long long v[kMaxFold];
#pragma unroll
  for (int j = 0; j < kMaxFold; ++j) v[j] = j < k ? spread[lane * k + j] : 0ull;
#pragma unroll
  for (int j = 0; j < kMaxFold; ++j) {
    if (j >= k) break;
    spread[lane * k + j] = 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v[j] += __shfl_xor(v[j], off, kWaveLanes);
    if (lane == 0) out[j] = accumulate ? out[j] + v[j] : v[j];
  }
}

// The captured step's epilogue in one launch (N07/N09/X04): fold the batch's spread
// counters into out[] (copied: no zero-fill node before the batch), advance the
// cursor's slot/id bases past it, and stamp the next step's time base from the
// device wall clock — three single-wave nodes (fill, fold, advance) plus the next
// step's clock node become one.  `cursor` is int64[4]: [3] keeps the time base
// of the batch that just ran.
__global__ __launch_bounds__(kWaveLanes) void pipeline_epilogue_kernel(unsigned long long* spread,
                                                                       unsigned long long* out, int k, int64_t* cursor,
                                                                       int64_t n, int64_t capacity, int64_t base_us,
                                                                       int64_t base_clk, int64_t rate_khz) {
  const int lane = threadIdx.x;
  if (spread != nullptr) {
    unsigned long long v[kMaxFold];
#pragma unroll
    for (int j = 0; j < kMaxFold; ++j) v[j] = j < k ? spread[lane * k + j] : 0ull;
#pragma unroll
    for (int j = 0; j < kMaxFold; ++j) {
      if (j >= k) break;
      spread[lane * k + j] = 0;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v[j] += __shfl_xor(v[j], off, kWaveLanes);
      if (lane == 0) out[j] = v[j];
    }
  }
  if (lane == 0) {
    cursor[0] = (cursor[0] + n) % capacity;
    cursor[1] += 3 * n;
    const int64_t ticks = static_cast<int64_t>(wall_clock64()) - base_clk;
    cursor[3] = cursor[2];  // the time base the finished batch used (PipelineGraph.last_batch)
    cursor[2] = base_us + ticks * 1000 / rate_khz;
  }
}

void launch_pipeline_epilogue(unsigned long long* spread, unsigned long long* out, int k, int64_t* cursor, int64_t n,
                              int64_t capacity, int64_t base_us, int64_t base_clk, int64_t rate_khz, hipStream_t s) {
  if (spread != nullptr && (k <= 0 || k > kMaxFold)) throw std::invalid_argument("pipeline epilogue: k out of range");
  if (capacity <= 0 || rate_khz <= 0) throw std::invalid_argument("pipeline epilogue: bad capacity / clock rate");
  hipLaunchKernelGGL(pipeline_epilogue_kernel, dim3(1), dim3(kWaveLanes), 0, s, spread, out, k, cursor, n, capacity,
                     base_us, base_clk, rate_khz);
  check_hip(hipGetLastError(), "pipeline_epilogue_kernel");
}

void launch_spread_fold(unsigned long long* spread, unsigned long long* out, int k, bool accumulate, hipStream_t s) {
  if (k <= 0 || k > kMaxFold) throw std::invalid_argument("spread fold: k out of range");
  hipLaunchKernelGGL(spread_fold_kernel, dim3(1), dim3(kWaveLanes), 0, s, spread, out, k, accumulate ? 1 : 0);
  check_hip(hipGetLastError(), "spread_fold_kernel");
}

void launch_pipeline_clock(int64_t* cursor, int64_t base_us, int64_t base_clk, int64_t rate_khz, hipStream_t s) {
  if (rate_khz <= 0) throw std::invalid_argument("wall clock rate must be positive");
  hipLaunchKernelGGL(pipeline_clock_kernel, dim3(1), dim3(1), 0, s, cursor, base_us, base_clk, rate_khz);
  check_hip(hipGetLastError(), "pipeline_clock_kernel");
}

void launch_pipeline_advance(int64_t* cursor, int64_t n, int64_t capacity, hipStream_t s) {
  if (capacity <= 0) throw std::invalid_argument("capacity must be positive");
  hipLaunchKernelGGL(pipeline_advance_kernel, dim3(1), dim3(1), 0, s, cursor, n, capacity);
  check_hip(hipGetLastError(), "pipeline_advance_kernel");
}

int64_t device_wall_clock(int device) {
  check_hip(hipSetDevice(device), "hipSetDevice");
  int64_t* d = nullptr;
  check_hip(hipMalloc(&d, sizeof(int64_t)), "hipMalloc");
  hipLaunchKernelGGL(wall_clock_kernel, dim3(1), dim3(1), 0, nullptr, d);
  int64_t v = 0;
  const hipError_t e1 = hipGetLastError();
  const hipError_t e2 = hipMemcpy(&v, d, sizeof(v), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  check_hip(e1, "wall_clock_kernel");
  check_hip(e2, "hipMemcpy wall clock");
  return v;
}

int64_t device_wall_clock_rate_khz(int device) {
  int rate = 0;
  check_hip(hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, device), "wall clock rate");
  return rate;
}

}  // namespace ahv

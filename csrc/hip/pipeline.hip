// Batched governance pipeline kernel (gfx950) and its host twin.
//
// Geometry: one wave (64 lanes) per workgroup, one session per lane, a
// 3-block LDS message window per wave (ahv/wave_sink.h: 12.5 KiB for 3
// blocks → 12 waves per CU, 3 per SIMD).  The SHA rounds are pure VALU
// (v_alignbit / v_bitop3 / v_add3); a wave alone issues a VALU op every 4
// cycles against the SIMD's 2, so ≥2 waves per SIMD keep the issue slots busy
// (measured SHA-256 ceiling: scripts/exp/sha_sol.hip).  A launch of n sessions is
// ⌈n/64⌉ workgroups: the 256 CUs are saturated from ~200k sessions per batch.
// There is no inter-workgroup data reuse, so no XCD remapping is needed.
//
// Batch counters (collective X04 input) are reduced across the wave with DPP
// shuffles and added with one 64-bit atomic per counter per wave.
#include <cstdlib>

#include "ahv/launch.h"
#include "ahv/pipeline.h"
#include "ahv/wave_sink.h"

namespace ahv {

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWaveLanes);
  return v;
}

// (64 threads, ≥MinWaves waves per SIMD).  The LDS window caps residency (8.4 KiB
// for 2 blocks → 4 waves per SIMD; 12.5 KiB for 3 blocks → 3), so MinWaves
// matches it: the VGPR budget is 128 or 168 registers.  Both shapes are
// instantiated; AHV_PIPE_WIN=2|3 selects one for A/B runs.
template <int MinWaves, int WinBlocks>
__global__ __launch_bounds__(kWaveLanes, MinWaves) void governance_pipeline_kernel(PipelineArgs a) {
  const uint32_t lane = threadIdx.x;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kWaveLanes + lane;
  PipeCounters c{};
  if (i < a.n) {
    WordWindowSink<WinBlocks> sink;
    sink.g_win = win_lds<WinBlocks>();
    sink.lane = lane;
    c = pipeline_session(a, i, sink);
  }
  if (a.stats) {
#pragma unroll
    for (int k = 0; k < kPipeStats; ++k) {
      const uint32_t s = wave_sum(c.v[k]);
      if (lane == 0 && s)
        atomicAdd(a.stats + (blockIdx.x % kStatSpread) * kPipeStats + k, static_cast<unsigned long long>(s));
    }
  }
  if (a.ev.cursor) {
    // one 64-bit atomic reserves the whole wave's records; lanes write at their
    // exclusive prefix offset
    const uint32_t nev = i < a.n ? pipeline_event_count(a, i, c) : 0u;
    uint32_t incl = nev;
#pragma unroll
    for (int off = 1; off < kWaveLanes; off <<= 1) {
      const uint32_t y = __shfl_up(incl, off, kWaveLanes);
      if (lane >= static_cast<uint32_t>(off)) incl += y;
    }
    const uint32_t total = __shfl(incl, kWaveLanes - 1, kWaveLanes);
    const int seg = static_cast<int>(blockIdx.x % kStatSpread);
    unsigned long long base = 0;
    if (lane == 0 && total) base = atomicAdd(a.ev.cursor + seg, static_cast<unsigned long long>(total));
    base = __shfl(base, 0, kWaveLanes);
    if (i < a.n) {
      const unsigned long long first = base + (incl - nev);
      pipeline_events(a, i, c, [&](uint32_t k, int64_t slot, const EventRec& e) {
        event_store(a.ev, seg, first + k, static_cast<int32_t>(slot), e);
      });
    }
  }
}

static int pipeline_window() {
  static const int w = [] {
    const char* e = std::getenv("AHV_PIPE_WIN");
    return e && std::atoi(e) == 2 ? 2 : 3;
  }();
  return w;
}

void launch_pipeline(const PipelineArgs& a, hipStream_t stream) {
  if (a.n <= 0) return;
  const int64_t blocks = (a.n + kWaveLanes - 1) / kWaveLanes;
  const dim3 grid(static_cast<uint32_t>(blocks)), block(kWaveLanes);
  if (pipeline_window() == 2) hipLaunchKernelGGL((governance_pipeline_kernel<4, 2>), grid, block, 0, stream, a);
  else hipLaunchKernelGGL((governance_pipeline_kernel<3, 3>), grid, block, 0, stream, a);
  check_hip(hipGetLastError(), "governance_pipeline_kernel launch");
}

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

void pipeline_host(const PipelineArgs& a) {
  HostSink sink;
  for (int64_t i = 0; i < a.n; ++i) {
    const PipeCounters c = pipeline_session(a, i, sink);
    if (a.stats)
      for (int k = 0; k < kPipeStats; ++k) a.stats[k] += c.v[k];
    if (a.ev.cursor) {
      const int seg = static_cast<int>((i / kWaveLanes) % kStatSpread);  // the device's workgroup mapping
      const unsigned long long first = a.ev.cursor[seg];
      a.ev.cursor[seg] += pipeline_event_count(a, i, c);
      pipeline_events(a, i, c, [&](uint32_t k, int64_t slot, const EventRec& e) {
        event_store(a.ev, seg, first + k, static_cast<int32_t>(slot), e);
      });
    }
  }
}


void kernels_pipeline(std::vector<KernelEntry>& out) {
  out.push_back({"governance_pipeline_kernel<3,3>", reinterpret_cast<const void*>(&governance_pipeline_kernel<3, 3>)});
  out.push_back({"governance_pipeline_kernel<4,2>", reinterpret_cast<const void*>(&governance_pipeline_kernel<4, 2>)});
}

}  // namespace ahv

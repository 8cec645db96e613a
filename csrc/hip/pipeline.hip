// Batched governance pipeline kernel (gfx950) and its host twin.
//
// Geometry: one wave (64 lanes) per workgroup, one session per lane, a 16 KiB LDS
// message ring per wave (ahv/wave_sink.h) → LDS allows 10 waves per CU; the SHA
// rounds are pure VALU (v_alignbit / v_bfi / v_add3), so ≥2 waves per SIMD keep
// the issue slots busy.  A launch of n sessions is ⌈n/64⌉ workgroups: the 256
// CUs are saturated from ~160k sessions per batch (10 waves × 256 CUs × 64).
// There is no inter-workgroup data reuse, so no XCD remapping is needed.
//
// Batch counters (collective X04 input) are reduced across the wave with DPP
// shuffles and added with one 64-bit atomic per counter per wave.
#include "ahv/launch.h"
#include "ahv/pipeline.h"
#include "ahv/wave_sink.h"

namespace ahv {

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWaveLanes);
  return v;
}

// (64 threads, ≥3 waves per SIMD): caps the allocation at 168 VGPRs, which this
// kernel meets without spilling — 12 waves per CU instead of 8.
__global__ __launch_bounds__(kWaveLanes, 3) void governance_pipeline_kernel(PipelineArgs a) {
  const uint32_t lane = threadIdx.x;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kWaveLanes + lane;
  PipeCounters c{};
  if (i < a.n) {
    WaveWindowSink sink;
    sink.lane = lane;
    c = pipeline_session(a, i, sink);
  }
  if (a.stats) {
#pragma unroll
    for (int k = 0; k < kPipeStats; ++k) {
      const uint32_t s = wave_sum(c.v[k]);
      if (lane == 0 && s) atomicAdd(a.stats + k, static_cast<unsigned long long>(s));
    }
  }
}

void launch_pipeline(const PipelineArgs& a, hipStream_t stream) {
  if (a.n <= 0) return;
  const int64_t blocks = (a.n + kWaveLanes - 1) / kWaveLanes;
  hipLaunchKernelGGL(governance_pipeline_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(kWaveLanes), 0,
                     stream, a);
  check_hip(hipGetLastError(), "governance_pipeline_kernel launch");
}

void pipeline_host(const PipelineArgs& a) {
  HostSink sink;
  for (int64_t i = 0; i < a.n; ++i) {
    const PipeCounters c = pipeline_session(a, i, sink);
    if (a.stats)
      for (int k = 0; k < kPipeStats; ++k) a.stats[k] += c.v[k];
  }
}

}  // namespace ahv

// Host-side declarations of kernel launchers and their CPU twins.
#pragma once

#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "ahv/hd.h"

namespace ahv {

inline void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

struct PipelineArgs;
void launch_pipeline(const PipelineArgs& a, hipStream_t stream);
void pipeline_host(const PipelineArgs& a);

}  // namespace ahv

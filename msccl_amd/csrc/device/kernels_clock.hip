// NPKit clock calibration (include/msccl_amd_npkit.h): the GPU's constant-rate clock, stored to
// host-mapped memory, lets the host place GPU timestamps on its own timeline.
#include <hip/hip_runtime.h>

#include "devcomm.h"

namespace msccl {

__global__ void clockProbeKernel(uint64_t* hostWord) {
  const uint64_t t = __builtin_amdgcn_s_memrealtime();
  __hip_atomic_store(hostWord, t, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int launchClockProbe(uint64_t* hostWord, void* stream) {
  hipLaunchKernelGGL(clockProbeKernel, dim3(1), dim3(1), 0, (hipStream_t)stream, hostWord);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // namespace msccl

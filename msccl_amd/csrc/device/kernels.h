// Kernel instantiation + host launch shim (one translation unit per element type so the
// 120 kernels build in parallel).
#pragma once
#include "interpreter.h"

namespace msccl {

// gridBlocks > 0: launch, returns 0 on success.  gridBlocks == kQueryResidency: returns how many
// workgroups of this kernel one CU holds at once (0 on error), which bounds a co-resident launch:
// every workgroup of a launch spins on others, so all of them must be resident together.
template <typename T, int OP, int PROTO>
int launchKernel(const LaunchArgs& args, int gridBlocks, void* stream) {
  if (gridBlocks == kQueryResidency) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, mscclKernel<T, OP, PROTO>, kNT, 0) != hipSuccess) return 0;
    return n;
  }
  hipLaunchKernelGGL((mscclKernel<T, OP, PROTO>), dim3(gridBlocks), dim3(kNT), 0, (hipStream_t)stream, args);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

#define MSCCL_DEFINE_TABLE(NAME, T)                                                                 \
  LaunchFn NAME[4][3] = {                                                                           \
      {launchKernel<T, kSum, pLL>, launchKernel<T, kSum, pLL128>, launchKernel<T, kSum, pSimple>},             \
      {launchKernel<T, kProd, pLL>, launchKernel<T, kProd, pLL128>, launchKernel<T, kProd, pSimple>},           \
      {launchKernel<T, kMax, pLL>, launchKernel<T, kMax, pLL128>, launchKernel<T, kMax, pSimple>},             \
      {launchKernel<T, kMin, pLL>, launchKernel<T, kMin, pLL128>, launchKernel<T, kMin, pSimple>}};

}  // namespace msccl

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

// the small-call kernel (mscclSmallKernel, LL): same contract as launchKernel; launches of at
// most kCompactLaunchRanks ranks take the variant with the compact argument block
template <typename T, int OP, int PROTO, int SET>
int launchSmallKernel(const LaunchArgs& args, int gridBlocks, void* stream) {
  constexpr int RC = kCompactLaunchRanks;
  if (gridBlocks == kQueryResidency) {
    int n = 0, m = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, mscclSmallKernel<T, OP, PROTO, kMaxLaunchRanks, SET>, kNT,
                                                     0) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&m, mscclSmallKernel<T, OP, PROTO, RC, SET>, kNT, 0) != hipSuccess)
      return 0;
    return n < m ? n : m;
  }
  if (args.nRanks <= RC) {
    LaunchArgsN<RC> a;
    a.nRanks = args.nRanks;
    a.pad = 0;
    for (int r = 0; r < RC; r++) a.w[r] = args.w[r];
    hipLaunchKernelGGL((mscclSmallKernel<T, OP, PROTO, RC, SET>), dim3(gridBlocks), dim3(kNT), 0, (hipStream_t)stream, a);
  } else {
    hipLaunchKernelGGL((mscclSmallKernel<T, OP, PROTO, kMaxLaunchRanks, SET>), dim3(gridBlocks), dim3(kNT), 0,
                       (hipStream_t)stream, args);
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// the flat tree's fold kernel (mscclFoldKernel, LL, Sum..Min): RankWork::nBlocks workgroups per rank
template <typename T, int OP>
int launchFoldKernel(const LaunchArgs& args, int gridBlocks, void* stream) {
  constexpr int RC = kCompactLaunchRanks;
  if (gridBlocks == kQueryResidency) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, mscclFoldKernel<T, OP, kMaxLaunchRanks>, kNT, 0) != hipSuccess)
      return 0;
    return n;
  }
  if (gridBlocks < args.nRanks) return 1;  // every rank has at least one workgroup
  if (args.nRanks <= RC) {
    LaunchArgsN<RC> a;
    a.nRanks = args.nRanks;
    a.pad = 0;
    for (int r = 0; r < RC; r++) a.w[r] = args.w[r];
    hipLaunchKernelGGL((mscclFoldKernel<T, OP, RC>), dim3(gridBlocks), dim3(kNT), 0, (hipStream_t)stream, a);
  } else {
    hipLaunchKernelGGL((mscclFoldKernel<T, OP, kMaxLaunchRanks>), dim3(gridBlocks), dim3(kNT), 0, (hipStream_t)stream,
                       args);
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// the two-phase fold (mscclTwoPhaseKernel, LL, Sum..Min): RankWork::nBlocks workgroups per rank
template <typename T, int OP>
int launchTwoPhaseKernel(const LaunchArgs& args, int gridBlocks, void* stream) {
  constexpr int RC = kCompactLaunchRanks;
  if (gridBlocks == kQueryResidency) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, mscclTwoPhaseKernel<T, OP, kMaxLaunchRanks>, kNT, 0) !=
        hipSuccess)
      return 0;
    return n;
  }
  if (gridBlocks < args.nRanks) return 1;
  if (args.nRanks <= RC) {
    LaunchArgsN<RC> a;
    a.nRanks = args.nRanks;
    a.pad = 0;
    for (int r = 0; r < RC; r++) a.w[r] = args.w[r];
    hipLaunchKernelGGL((mscclTwoPhaseKernel<T, OP, RC>), dim3(gridBlocks), dim3(kNT), 0, (hipStream_t)stream, a);
  } else {
    hipLaunchKernelGGL((mscclTwoPhaseKernel<T, OP, kMaxLaunchRanks>), dim3(gridBlocks), dim3(kNT), 0,
                       (hipStream_t)stream, args);
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// the direct form (mscclDirectKernel, Simple schedules, Sum..Min): every rank of the communicator in
// the launch, RankWork in rank order
template <typename T, int OP>
int launchDirectKernel(const LaunchArgs& args, int gridBlocks, void* stream) {
  constexpr int RC = kCompactLaunchRanks;
  if (gridBlocks == kQueryResidency) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, mscclDirectKernel<T, OP, kMaxLaunchRanks>, kNT, 0) != hipSuccess)
      return 0;
    return n;
  }
  if (gridBlocks < args.nRanks) return 1;
  if (args.nRanks <= RC) {
    LaunchArgsN<RC> a;
    a.nRanks = args.nRanks;
    a.pad = 0;
    for (int r = 0; r < RC; r++) a.w[r] = args.w[r];
    hipLaunchKernelGGL((mscclDirectKernel<T, OP, RC>), dim3(gridBlocks), dim3(kNT), 0, (hipStream_t)stream, a);
  } else {
    hipLaunchKernelGGL((mscclDirectKernel<T, OP, kMaxLaunchRanks>), dim3(gridBlocks), dim3(kNT), 0,
                       (hipStream_t)stream, args);
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// the pair kernel (mscclPairKernel, LL, Sum..Min): same contract as launchSmallKernel
template <typename T, int OP>
int launchPairKernel(const LaunchArgs& args, int gridBlocks, void* stream) {
  constexpr int RC = kCompactLaunchRanks;
  if (gridBlocks == kQueryResidency) {
    int n = 0, m = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, mscclPairKernel<T, OP, kMaxLaunchRanks>, kNT, 0) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&m, mscclPairKernel<T, OP, RC>, kNT, 0) != hipSuccess)
      return 0;
    return n < m ? n : m;
  }
  if (args.nRanks <= RC) {
    LaunchArgsN<RC> a;
    a.nRanks = args.nRanks;
    a.pad = 0;
    for (int r = 0; r < RC; r++) a.w[r] = args.w[r];
    hipLaunchKernelGGL((mscclPairKernel<T, OP, RC>), dim3(gridBlocks), dim3(kNT), 0, (hipStream_t)stream, a);
  } else {
    hipLaunchKernelGGL((mscclPairKernel<T, OP, kMaxLaunchRanks>), dim3(gridBlocks), dim3(kNT), 0, (hipStream_t)stream,
                       args);
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// nRanks == 1 with a user PreMulSum op: dst = src * scale (the reference's oneRankReduce,
// onerank_reduce.cu:12-44: ReduceOrCopyMulti with the preOp applied, postOp identity).
template <typename T>
__global__ void __launch_bounds__(256) oneRankScaleKernel(const T* src, T* dst, size_t n, uint64_t arg, int argIsPtr) {
  if (argIsPtr) {
    T x;
    __builtin_memcpy(&x, (const void*)arg, sizeof(T));
    arg = 0;
    __builtin_memcpy(&arg, &x, sizeof(T));
  }
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = scaleElem<T>(src[i], arg);
}

template <typename T>
int launchOneRankScale(const void* src, void* dst, size_t n, uint64_t arg, int argIsPtr, void* stream) {
  const size_t blocks = n == 0 ? 1 : (n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048;
  hipLaunchKernelGGL((oneRankScaleKernel<T>), dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, (const T*)src,
                     (T*)dst, n, arg, argIsPtr);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// [op][protocol]: Sum, Prod, Max, Min, PreMulSum, SumPostDiv x LL, LL128, Simple.  PreMulSum and
// SumPostDiv only run in the ring fallback (LL or Simple); SumPostDiv exists for integer types.
#define MSCCL_OPS_0_3(T)                                                                                   \
  {launchKernel<T, kSum, pLL>, launchKernel<T, kSum, pLL128>, launchKernel<T, kSum, pSimple>},             \
      {launchKernel<T, kProd, pLL>, launchKernel<T, kProd, pLL128>, launchKernel<T, kProd, pSimple>},      \
      {launchKernel<T, kMax, pLL>, launchKernel<T, kMax, pLL128>, launchKernel<T, kMax, pSimple>},         \
      {launchKernel<T, kMin, pLL>, launchKernel<T, kMin, pLL128>, launchKernel<T, kMin, pSimple>},         \
      {launchKernel<T, kPreMulSum, pLL>, nullptr, launchKernel<T, kPreMulSum, pSimple>}
// Small-call kernels: MSCCL schedules (ops Sum..Min) on LL.
#define MSCCL_SMALL(NAME, T)                                                                               \
  LaunchFn NAME##_small[2][4] = {                                                                          \
      {launchSmallKernel<T, kSum, pLL, kSetAll>, launchSmallKernel<T, kProd, pLL, kSetAll>,                 \
       launchSmallKernel<T, kMax, pLL, kSetAll>, launchSmallKernel<T, kMin, pLL, kSetAll>},                 \
      {launchSmallKernel<T, kSum, pLL, kSetExchange>, launchSmallKernel<T, kProd, pLL, kSetExchange>,       \
       launchSmallKernel<T, kMax, pLL, kSetExchange>, launchSmallKernel<T, kMin, pLL, kSetExchange>}};      \
  LaunchFn NAME##_fold[4] = {launchFoldKernel<T, kSum>, launchFoldKernel<T, kProd>, launchFoldKernel<T, kMax>, \
                             launchFoldKernel<T, kMin>};                                                   \
  LaunchFn NAME##_pair[4] = {launchPairKernel<T, kSum>, launchPairKernel<T, kProd>, launchPairKernel<T, kMax>, \
                             launchPairKernel<T, kMin>};                                                   \
  LaunchFn NAME##_two[4] = {launchTwoPhaseKernel<T, kSum>, launchTwoPhaseKernel<T, kProd>,                  \
                            launchTwoPhaseKernel<T, kMax>, launchTwoPhaseKernel<T, kMin>};                 \
  LaunchFn NAME##_direct[4] = {launchDirectKernel<T, kSum>, launchDirectKernel<T, kProd>,                   \
                               launchDirectKernel<T, kMax>, launchDirectKernel<T, kMin>};                  \
  extern const uint32_t NAME##_layout = kWorkLayout;
#define MSCCL_DEFINE_TABLE(NAME, T)                                                                        \
  LaunchFn NAME[6][3] = {MSCCL_OPS_0_3(T),                                                                 \
                         {launchKernel<T, kSumPostDiv, pLL>, nullptr, launchKernel<T, kSumPostDiv, pSimple>}}; \
  MSCCL_SMALL(NAME, T)                                                                                     \
  OneRankFn NAME##_one = launchOneRankScale<T>;
#ifndef MSCCL_SMALL_ONLY
#define MSCCL_DEFINE_TABLE_FP(NAME, T)                                                                     \
  LaunchFn NAME[6][3] = {MSCCL_OPS_0_3(T), {nullptr, nullptr, nullptr}};                                   \
  MSCCL_SMALL(NAME, T)                                                                                     \
  OneRankFn NAME##_one = launchOneRankScale<T>;
#else
// measurement builds of one type's small-call and fold kernels only (tools/varbuild.sh): the
// general kernel is not compiled, calls that need it fail to launch
#define MSCCL_DEFINE_TABLE_FP(NAME, T)                                                                     \
  LaunchFn NAME[6][3] = {};                                                                                \
  MSCCL_SMALL(NAME, T)                                                                                     \
  OneRankFn NAME##_one = launchOneRankScale<T>;
#endif

}  // namespace msccl

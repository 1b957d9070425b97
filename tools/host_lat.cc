// Host-side cost of one grouped AllReduce over co-resident ranks, from C (no Python):
//   tools/host_lat [ranks] [bytes] [iters] [null stream 0/1] [host gap us]
// prints the host time per group call and the stream time per launch, plus the same for an
// empty kernel launch (the HIP launch floor).  Build:
//   hipcc -O2 --offload-arch=gfx950 -Iinclude tools/host_lat.cc -o tools/host_lat -Lmsccl_amd -lmsccl_amd \
//     -Wl,-rpath,'$ORIGIN/../msccl_amd'
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include <vector>

#include "nccl.h"

__global__ void emptyKernel(int) {}
struct BigArgs { char b[4000]; };
__global__ void emptyBigKernel(BigArgs) {}  // the interpreter's kernel-argument size

static double now() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 2;
  const size_t bytes = argc > 2 ? strtoull(argv[2], nullptr, 10) : 128;
  const int iters = argc > 3 ? atoi(argv[3]) : 2000;
  const int nullStream = argc > 4 ? atoi(argv[4]) : 0;     // 1: launch on the null stream
  const double gapUs = argc > 5 ? atof(argv[5]) : 0.0;    // host spin between calls (idle GPU)
  std::vector<int> devs(n, 0);
  std::vector<ncclComm_t> comms(n);
  if (ncclCommInitAll(comms.data(), n, devs.data()) != ncclSuccess) return 1;
  std::vector<float*> bufs(n);
  for (auto& b : bufs) hipMalloc(&b, bytes + 64);
  hipStream_t s = nullptr;
  if (!nullStream) hipStreamCreate(&s);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto step = [&]() {
    ncclGroupStart();
    for (int r = 0; r < n; r++) ncclAllReduce(bufs[r], bufs[r], bytes / 4, ncclFloat32, ncclSum, comms[r], s);
    return ncclGroupEnd();
  };
  for (int i = 0; i < 50; i++)
    if (step() != ncclSuccess) return 2;
  hipStreamSynchronize(s);
  hipEventRecord(e0, s);
  double t0 = now();
  for (int i = 0; i < iters; i++) {
    step();
    if (gapUs > 0)
      for (double t = now(); now() - t < gapUs * 1e-6;) {
      }
  }
  double host = (now() - t0) / iters;
  hipEventRecord(e1, s);
  hipStreamSynchronize(s);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  printf("allreduce %zu B x%d ranks: host %.2f us per group call, stream %.2f us per launch\n", bytes, n, host * 1e6,
         ms * 1e3 / iters);
  for (int i = 0; i < 50; i++) hipLaunchKernelGGL(emptyKernel, dim3(1), dim3(64), 0, s, 0);
  hipStreamSynchronize(s);
  hipEventRecord(e0, s);
  t0 = now();
  for (int i = 0; i < iters; i++) hipLaunchKernelGGL(emptyKernel, dim3(1), dim3(64), 0, s, 0);
  host = (now() - t0) / iters;
  hipEventRecord(e1, s);
  hipStreamSynchronize(s);
  hipEventElapsedTime(&ms, e0, e1);
  printf("empty kernel: host %.2f us per launch, stream %.2f us per launch\n", host * 1e6, ms * 1e3 / iters);
  BigArgs big = {};
  for (int i = 0; i < 50; i++) hipLaunchKernelGGL(emptyBigKernel, dim3(1), dim3(64), 0, s, big);
  hipStreamSynchronize(s);
  hipEventRecord(e0, s);
  t0 = now();
  for (int i = 0; i < iters; i++) hipLaunchKernelGGL(emptyBigKernel, dim3(1), dim3(64), 0, s, big);
  host = (now() - t0) / iters;
  hipEventRecord(e1, s);
  hipStreamSynchronize(s);
  hipEventElapsedTime(&ms, e0, e1);
  printf("empty kernel, 4000-B arguments: host %.2f us per launch, stream %.2f us per launch\n", host * 1e6,
         ms * 1e3 / iters);
  for (auto c : comms) ncclCommDestroy(c);
  return 0;
}

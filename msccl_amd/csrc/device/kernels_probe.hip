// 16-B line atomicity probe (include/msccl_amd.h: mscclAmdLineTearProbe).
//
// The CDNA4 LL128 form (interpreter.h: l16Op) guards 12 payload bytes with a 4-B flag in the same
// 16-B line; it is correct only if a receiver never observes a line whose flag is new and whose
// payload is old (or mixed).  The reference enables LL128 only where its line atomicity holds
// (tuning.cc:210-214).  Here writers on one device stream 16-B lines {d0(k,l), d1(k,l), d2(k,l), k}
// into another device's uncached memory (the FIFO memory of transport.cc) for k = 1..iters, while
// readers on the receiving device poll the same lines with the FIFO's 16-B loads and count every
// observed line whose dwords do not belong to one k ("torn").
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "devcomm.h"

namespace msccl {

typedef uint32_t p32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ p32x4 probeLine(uint32_t k, uint32_t l) {
  const uint32_t a = k * 0x01000193u ^ (l * 0x9E3779B1u);
  return (p32x4){a, ~a, a + 0x5bd1e995u, k};
}

// Each thread owns lines l = tid + j * nthreadsTotal; iteration k rewrites all of them.
__global__ void __launch_bounds__(256) lineWriterKernel(p32x4* lines, int nLines, int iters) {
  const int stride = gridDim.x * blockDim.x;
  for (int k = 1; k <= iters; k++)
    for (int l = blockIdx.x * blockDim.x + threadIdx.x; l < nLines; l += stride) {
      const p32x4 v = probeLine((uint32_t)k, (uint32_t)l);
      asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(lines + l), "v"(v) : "memory");
    }
}

// Readers poll their lines until each shows k == iters or `ticks` (100 MHz) pass: every wave ends.
// out[0] += lines observed with a flag, out[1] += torn lines, out[2] = lines that reached iters.
__global__ void __launch_bounds__(256) lineReaderKernel(const p32x4* lines, int nLines, int iters, uint64_t ticks,
                                                        unsigned long long* out) {
  const int stride = gridDim.x * blockDim.x;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long seen = 0, torn = 0, done = 0;
  for (int l = blockIdx.x * blockDim.x + threadIdx.x; l < nLines; l += stride) {
    while (true) {
      p32x4 v;
      asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(v) : "v"(lines + l) : "memory");
      if (v.w != 0) {
        seen++;
        const p32x4 e = probeLine(v.w, (uint32_t)l);
        if (v.x != e.x || v.y != e.y || v.z != e.z) torn++;
      }
      if (v.w == (uint32_t)iters) {
        done++;
        break;
      }
      if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) break;
    }
  }
  atomicAdd(out + 0, seen);
  atomicAdd(out + 1, torn);
  atomicAdd(out + 2, done);
}

int launchLineWriter(void* lines, int nLines, int iters, int blocks, void* stream) {
  hipLaunchKernelGGL(lineWriterKernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (p32x4*)lines, nLines,
                     iters);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int launchLineReader(const void* lines, int nLines, int iters, uint64_t ticks, unsigned long long* out, int blocks,
                     void* stream) {
  hipLaunchKernelGGL(lineReaderKernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const p32x4*)lines,
                     nLines, iters, ticks, out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // namespace msccl

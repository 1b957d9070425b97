// Standalone check of the 16-B pack functors and buffer load/store helpers.
#include <stdio.h>
#include "../msccl_amd/csrc/device/primitives.h"
using namespace msccl;
__global__ void k(const float* a, const float* b, float* o, int n) {
  int p = threadIdx.x;
  __amdgpu_buffer_rsrc_t ra = makeRsrc(a), rb = makeRsrc(b), ro = makeRsrc(o);
  u32x4 x = ld16<kAuxLocal>(ra, p * 16), y = ld16<kAuxLocal>(rb, p * 16);
  st16<kAuxLocal>(ro, p * 16, Fn<float, kSum>::pack(x, y));
}
int main() {
  const int n = 256;
  float ha[n], hb[n], ho[n];
  for (int i = 0; i < n; i++) { ha[i] = i; hb[i] = 1000 * i; }
  float *da, *db, *dout;
  hipMalloc(&da, n * 4); hipMalloc(&db, n * 4); hipMalloc(&dout, n * 4);
  hipMemcpy(da, ha, n * 4, hipMemcpyHostToDevice); hipMemcpy(db, hb, n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(n / 4), 0, 0, da, db, dout, n);
  hipMemcpy(ho, dout, n * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; i++) if (ho[i] != ha[i] + hb[i]) { if (bad < 8) printf("i=%d got %f want %f\n", i, ho[i], ha[i] + hb[i]); bad++; }
  printf("pack test: %d bad\n", bad);
  return bad != 0;
}

/* nccl-tests-style C caller of libmsccl_amd.so: compiled against include/nccl.h exactly as a
 * program written for the reference's nccl.h would be (cudaStream_t -> hipStream_t).
 *
 *   c_allreduce NRANKS COUNT [--version-only]
 *
 * Creates NRANKS communicators with ncclCommInitAll (all on device 0 unless MSCCL_AMD_DEVS="0,1,..."),
 * runs one in-place float Sum AllReduce per rank inside ncclGroupStart/End and checks every element
 * equals 1+2+..+NRANKS.  MSCCL_XML_FILES must name a matching schedule.  Exit code 0 = pass. */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nccl.h"

#define CHECK(cmd)                                                                              \
  do {                                                                                          \
    ncclResult_t r_ = (cmd);                                                                    \
    if (r_ != ncclSuccess) {                                                                    \
      fprintf(stderr, "%s:%d %s -> %s (%s)\n", __FILE__, __LINE__, #cmd, ncclGetErrorString(r_), \
              ncclGetLastError(NULL));                                                          \
      return 1;                                                                                 \
    }                                                                                           \
  } while (0)

int main(int argc, char** argv) {
  int version = 0;
  CHECK(ncclGetVersion(&version));
  printf("nccl version code %d\n", version);
  if (argc > 3 && strcmp(argv[3], "--version-only") == 0) return 0;
  int n = argc > 1 ? atoi(argv[1]) : 2;
  size_t count = argc > 2 ? (size_t)atol(argv[2]) : (size_t)1 << 20;
  if (n < 1 || n > 16) return 2;
  int devs[16] = {0};
  const char* dl = getenv("MSCCL_AMD_DEVS");
  for (int i = 0; dl && i < n; i++) {
    devs[i] = atoi(dl);
    dl = strchr(dl, ',');
    if (dl) dl++;
  }
  ncclComm_t comms[16];
  CHECK(ncclCommInitAll(comms, n, devs));
  float* buf[16];
  hipStream_t st[16];
  float* host = (float*)malloc(count * sizeof(float));
  for (int r = 0; r < n; r++) {
    if (hipSetDevice(devs[r]) != hipSuccess || hipMalloc((void**)&buf[r], count * sizeof(float)) != hipSuccess ||
        hipStreamCreate(&st[r]) != hipSuccess)
      return 3;
    for (size_t i = 0; i < count; i++) host[i] = (float)(r + 1);
    if (hipMemcpy(buf[r], host, count * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) return 3;
  }
  CHECK(ncclGroupStart());
  for (int r = 0; r < n; r++) CHECK(ncclAllReduce(buf[r], buf[r], count, ncclFloat, ncclSum, comms[r], st[r]));
  CHECK(ncclGroupEnd());
  int bad = 0;
  const float want = (float)(n * (n + 1) / 2);
  for (int r = 0; r < n; r++) {
    if (hipSetDevice(devs[r]) != hipSuccess || hipStreamSynchronize(st[r]) != hipSuccess) return 3;
    ncclResult_t ae;
    CHECK(ncclCommGetAsyncError(comms[r], &ae));
    if (ae != ncclSuccess) bad++;
    if (hipMemcpy(host, buf[r], count * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) return 3;
    for (size_t i = 0; i < count; i++)
      if (host[i] != want) {
        if (bad < 5) fprintf(stderr, "rank %d element %zu = %g, want %g\n", r, i, host[i], want);
        bad++;
        break;
      }
    hipFree(buf[r]);
    hipStreamDestroy(st[r]);
    CHECK(ncclCommDestroy(comms[r]));
  }
  free(host);
  printf("%s: %d ranks x %zu floats\n", bad ? "FAIL" : "PASS", n, count);
  return bad ? 1 : 0;
}

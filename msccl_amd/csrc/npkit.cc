// NPKit-compatible event log: device buffers, host/GPU clock calibration and the dump
// (include/msccl_amd_npkit.h).  Replaces the reference's NpKit class (src/misc/npkit.cc:31-174):
//   * buffers are per communicator (the reference's are per process) and live in device memory
//     for the communicator's lifetime, one per thread block;
//   * the host time of each launch start comes from a calibration of the GPU's constant-rate
//     clock against the host clock at init, instead of a host thread that rewrites a
//     host-mapped counter for ever (one CPU core per process in the reference);
//   * the dump writes the reference's file set, so its trace generator reads it unchanged.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "../../include/msccl_amd_npkit.h"
#include "comm.h"
#include "debug.h"

namespace msccl {

namespace {

ncclResult_t hipErr(hipError_t e, const char* what) {
  if (e == hipSuccess) return ncclSuccess;
  WARN("%s failed: %s", what, hipGetErrorString(e));
  return ncclUnhandledCudaError;
}

int64_t hostNs() {  // the reference's CPU timestamp: system_clock nanoseconds (npkit.cc:21-29)
  return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::system_clock::now().time_since_epoch())
      .count();
}

// Offset such that host ns = npkitTicksToNs(ticks, khz) + offset.  The probe kernel stores the GPU clock
// to host-mapped memory; the host sees it at most a PCIe write later, so every sample
// over-estimates the offset by that latency and the smallest sample is kept.
ncclResult_t calibrate(int khz, int64_t* offset) {
  uint64_t* word = nullptr;
  NCCLCHECK(hipErr(hipHostMalloc((void**)&word, 64, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc"));
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
    hipHostFree(word);
    return ncclUnhandledCudaError;
  }
  int64_t best = INT64_MAX;
  ncclResult_t res = ncclSuccess;
  for (int i = 0; i < 16 && res == ncclSuccess; i++) {
    __atomic_store_n(word, 0ull, __ATOMIC_RELEASE);
    if (launchClockProbe(word, (void*)s) != 0) {
      res = ncclUnhandledCudaError;
      break;
    }
    uint64_t t;
    const int64_t deadline = hostNs() + 5000000000ll;
    while ((t = __atomic_load_n(word, __ATOMIC_ACQUIRE)) == 0) {
      if (hostNs() > deadline) {
        res = ncclSystemError;
        break;
      }
    }
    if (res != ncclSuccess) break;
    const int64_t seen = hostNs();
    best = std::min(best, seen - npkitTicksToNs(t, khz));
    hipStreamSynchronize(s);
  }
  hipStreamSynchronize(s);
  hipStreamDestroy(s);
  hipHostFree(word);
  if (res == ncclSuccess) *offset = best;
  return res;
}

bool writeFile(const std::string& path, const void* data, size_t bytes) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) return false;
  const bool ok = bytes == 0 || fwrite(data, 1, bytes, f) == bytes;
  return fclose(f) == 0 && ok;
}

}  // namespace

ncclResult_t npkitSetup(ncclComm* comm) {
  if (envInt("MSCCL_AMD_NPKIT", 0) <= 0) return ncclSuccess;
  const int64_t cap = std::max<int64_t>(16, std::min<int64_t>(1 << 20, envInt("MSCCL_AMD_NPKIT_EVENTS", 1 << 16)));
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, comm->cudaDev) != hipSuccess || khz <= 0) khz = 100000;
  NpkitLog lg;
  memset(&lg, 0, sizeof(lg));
  lg.cap = (int32_t)cap;
  lg.clockKHz = khz;
  NCCLCHECK(calibrate(khz, &lg.cpuOffsetNs));
  const size_t evBytes = (size_t)kNpkitDevBuffers * cap * sizeof(NpkitEvent);
  NCCLCHECK(hipErr(hipMalloc(&comm->dNpkitEvents, evBytes), "hipMalloc npkit events"));
  NCCLCHECK(hipErr(hipMalloc(&comm->dNpkitHeads, kNpkitDevBuffers * sizeof(uint64_t)), "hipMalloc npkit heads"));
  NCCLCHECK(hipErr(hipMemset(comm->dNpkitHeads, 0, kNpkitDevBuffers * sizeof(uint64_t)), "hipMemset"));
  lg.events = comm->dNpkitEvents;
  lg.heads = comm->dNpkitHeads;
  NCCLCHECK(hipErr(hipMalloc(&comm->dNpkit, sizeof(NpkitLog)), "hipMalloc npkit"));
  NCCLCHECK(hipErr(hipMemcpy(comm->dNpkit, &lg, sizeof(lg), hipMemcpyHostToDevice), "hipMemcpy"));
  comm->npkitCap = (int)cap;
  comm->npkitClockKHz = khz;
  INFO(kSubInit, "NPKit: %d buffers x %lld events, GPU clock %d kHz", kNpkitDevBuffers, (long long)cap, khz);
  return ncclSuccess;
}

// The file set of NpKit::Dump (npkit.cc:64-127), rank = the communicator's rank.
ncclResult_t npkitDump(ncclComm* comm, const char* dir) {
  if (!comm->dNpkit) return ncclInvalidUsage;
  std::string d = dir ? dir : (getenv("NPKIT_DUMP_DIR") ? getenv("NPKIT_DUMP_DIR") : "/tmp/");
  if (d.empty()) d = ".";
  if (d.back() != '/') d += '/';
  mkdir(d.c_str(), 0755);
  hipSetDevice(comm->cudaDev);
  NCCLCHECK(hipErr(hipDeviceSynchronize(), "hipDeviceSynchronize"));
  std::vector<uint64_t> heads(kNpkitDevBuffers);
  NCCLCHECK(hipErr(hipMemcpy(heads.data(), comm->dNpkitHeads, heads.size() * sizeof(uint64_t), hipMemcpyDeviceToHost),
                   "hipMemcpy"));
  const std::string r = std::to_string(comm->rank);
  std::vector<NpkitEvent> ev;
  bool ok = true;
  for (int b = 0; b < MSCCL_AMD_NPKIT_GPU_BUFFERS; b++) {
    size_t n = 0;
    if (b < kNpkitDevBuffers) n = (size_t)std::min<uint64_t>(heads[b], (uint64_t)comm->npkitCap);
    ev.resize(n);
    if (n)
      NCCLCHECK(hipErr(hipMemcpy(ev.data(), comm->dNpkitEvents + (size_t)b * comm->npkitCap, n * sizeof(NpkitEvent),
                                 hipMemcpyDeviceToHost), "hipMemcpy"));
    ok = ok && writeFile(d + "gpu_events_rank_" + r + "_buf_" + std::to_string(b), ev.data(), n * sizeof(NpkitEvent));
  }
  for (int c = 0; c < MSCCL_AMD_NPKIT_CPU_BUFFERS; c++)
    ok = ok && writeFile(d + "cpu_events_rank_" + r + "_channel_" + std::to_string(c), nullptr, 0);
  const std::string num = "1", den = "1000000000", khz = std::to_string(comm->npkitClockKHz);
  ok = ok && writeFile(d + "cpu_clock_period_num_rank_" + r, num.data(), num.size());
  ok = ok && writeFile(d + "cpu_clock_period_den_rank_" + r, den.data(), den.size());
  ok = ok && writeFile(d + "gpu_clock_rate_rank_" + r, khz.data(), khz.size());
  if (!ok) {
    WARN("NPKit: could not write the dump into %s", d.c_str());
    return ncclSystemError;
  }
  INFO(kSubInit, "NPKit: rank %d dumped into %s", comm->rank, d.c_str());
  return ncclSuccess;
}

void npkitFree(ncclComm* comm) {
  if (comm->dNpkit) hipFree(comm->dNpkit);
  if (comm->dNpkitEvents) hipFree(comm->dNpkitEvents);
  if (comm->dNpkitHeads) hipFree(comm->dNpkitHeads);
  comm->dNpkit = nullptr;
  comm->dNpkitEvents = nullptr;
  comm->dNpkitHeads = nullptr;
}

}  // namespace msccl

extern "C" int mscclAmdNpkitDump(ncclComm_t comm, const char* dir) {
  if (!msccl::commValid(comm)) return ncclInvalidArgument;
  return msccl::npkitDump(comm, dir);
}

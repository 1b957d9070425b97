// Communicator creation / destruction (reference init.cc:87-1255, single-node MSCCL subset).
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <mutex>
#include <thread>

#include <stdio.h>

#include <algorithm>

#include "bootstrap.h"
#include "comm.h"
#include "debug.h"
#include "lower.h"
#include "group.h"
#include "plan.h"

using namespace msccl;

namespace msccl {

bool commValid(const ncclComm* comm) { return comm != nullptr && comm->magic == kCommMagic; }

namespace {

ncclResult_t hipErr(hipError_t e, const char* what) {
  if (e == hipSuccess) return ncclSuccess;
  WARN("%s failed: %s", what, hipGetErrorString(e));
  return ncclUnhandledCudaError;
}

// Load MSCCL_XML_FILES / MSCCL_CONFIG for this rank (init.cc:781-800).
ncclResult_t loadAlgos(ncclComm* comm) {
  const char* files = getenv("MSCCL_XML_FILES");
  const char* cfg = getenv("MSCCL_CONFIG");
  if (files) loadAlgosFromXmlFiles(files, &comm->algos, kMaxChannels, comm->rank, comm->nRanks);
  if (cfg) NCCLCHECK(loadAlgosFromConfig(cfg, &comm->algos, &comm->regs, kMaxChannels, comm->rank, comm->nRanks));
  return ncclSuccess;
}

// One-hop AllReduce schedules (lower.cc): every rank loads each LL AllReduce schedule once per
// rank of the communicator (as each of them loads it) and decides the same; the init allgather
// then keeps a lowering only where every rank reached it (applySplits).
void analyzeLowering(ncclComm* comm) {
  comm->algoFold.assign(comm->algos.size(), ncclComm::FoldProgram());
  comm->algoDirect.assign(comm->algos.size(), ncclComm::DirectProgram());
  if (comm->knobs.direct && lowerOffered()) {
    // the direct form of Simple schedules (lower.h: DirectLowering); used only when every rank of
    // the communicator runs in one launch (enqueue.cc: launchGroup)
    for (size_t g = 0; g < comm->algos.size(); g++) {
      const Algorithm& a = comm->algos[g];
      if (!a.valid || a.proto != kProtoSimple || a.path.empty() || a.ngpus != comm->nRanks ||
          !(a.coll == kAllReduce || a.coll == kReduceScatter || a.coll == kAllGather))
        continue;
      const DirectLowering dl = directScheduleFile(a.path, comm->nRanks);
      if (dl.ok) {
        ncclComm::DirectProgram& d = comm->algoDirect[g];
        d.coll = dl.coll;
        d.chunkClass = dl.chunkClass;
        for (auto& perRank : dl.order) d.order.push_back(perRank[comm->rank]);
      }
      INFO(kSubInit, "MSCCL: algorithm %s %s", a.name.c_str(),
           dl.ok ? "has a direct form (ranks in one launch write each other's buffers)"
                 : ("has no direct form (" + dl.why + ")").c_str());
    }
  }
  if (!comm->knobs.lower || !flatEnabled(comm) || !lowerOffered()) return;
  for (size_t g = 0; g < comm->algos.size(); g++) {
    const Algorithm& a = comm->algos[g];
    // a schedule for another rank count is never selected (selectAlgo): nothing to decide
    if (!a.valid || a.coll != kAllReduce || a.proto != kProtoLL || a.path.empty() || a.ngpus != comm->nRanks) continue;
    const FoldLowering fl = lowerScheduleFile(a.path, comm->nRanks);
    if (fl.ok) {
      ncclComm::FoldProgram& f = comm->algoFold[g];
      f.chunkClass = fl.chunkClass;
      for (auto& perRank : fl.order) f.order.push_back(perRank[comm->rank]);
      if (fl.twoPhase) f.owner = fl.owner;
    }
    INFO(kSubInit, "MSCCL: algorithm %s %s%s", a.name.c_str(),
         fl.ok ? "is a one-hop fold: calls up to MSCCL_AMD_LOWER_MAX_BYTES run the fold kernel"
               : ("runs interpreted (" + fl.why + ")").c_str(),
         !fl.ok ? "" : fl.twoPhase ? "; larger calls run its two-phase form" : (", not two-phase: " + fl.whyNotTwoPhase).c_str());
  }
}

// Per-rank device state that does not depend on peers.
ncclResult_t commLocalSetup(ncclComm* comm) {
  NCCLCHECK(hipErr(hipSetDevice(comm->cudaDev), "hipSetDevice"));
  if (const char* stale = kernelLayoutMismatch()) {
    WARN("MSCCL: the %s kernels were built with another RankWork layout than the host code (a stale kernel "
         "object: rebuild the library)", stale);
    return ncclInternalError;
  }
  if (comm->nRanks > 1) NCCLCHECK(loadAlgos(comm));
  // 0 (default) = waits never time out, as in the reference; > 0 bounds every single wait
  comm->timeoutSec = (double)std::max<int64_t>(0, envInt("MSCCL_AMD_TIMEOUT_SEC", 0));
  comm->timeoutTicks = (uint64_t)(comm->timeoutSec * 1e8);  // s_memrealtime runs at 100 MHz
  if (envInt("MSCCL_AMD_TEST_LL_CLEANUP", 0) != 0) {  // TEST_LL_CLEANUP (devcomm.h:56-63)
    comm->llFlagMask = 0xffu;
    comm->llCleanMask = 0x78u;
  }
  comm->knobs = Knobs::fromEnv();
  comm->ringFallback = comm->knobs.ringFallback != 0;
  analyzeLowering(comm);
  NCCLCHECK(hipErr(hipHostMalloc((void**)&comm->hostAbort, 64, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc"));
  NCCLCHECK(hipErr(hipHostMalloc((void**)&comm->hostErr, 64, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc"));
  *comm->hostAbort = 0;
  *comm->hostErr = 0;
  NCCLCHECK(hipErr(hipHostGetDevicePointer((void**)&comm->devAbort, comm->hostAbort, 0), "hipHostGetDevicePointer"));
  NCCLCHECK(hipErr(hipHostGetDevicePointer((void**)&comm->devErr, comm->hostErr, 0), "hipHostGetDevicePointer"));
  comm->workIndex = 1;  // flags start at 0 (init.cc:300-302)
  NCCLCHECK(hipErr(hipEventCreateWithFlags(&comm->doneEvent, hipEventDisableTiming), "hipEventCreate"));
  // scratch = max over algorithms of maxBytes * s_chunks / nchunksperloop (init.cc:809-835)
  size_t scratch = 0;
  for (auto& a : comm->algos)
    if (a.nchunksPerLoop > 0) {
      double need = (double)a.maxBytes * (double)a.nScratchChunks / (double)a.nchunksPerLoop;
      size_t s = need > 1.8e19 ? (size_t)-1 : (size_t)need;
      scratch = std::max(scratch, s);
    }
  size_t cap = (size_t)envInt("MSCCL_AMD_MAX_SCRATCH", (int64_t)8 << 30);
  if (scratch > cap) {
    INFO(kSubInit, "MSCCL scratch %zu bytes capped to %zu (MSCCL_AMD_MAX_SCRATCH)", scratch, cap);
    scratch = cap;
  }
  if (scratch > 0) {
    NCCLCHECK(hipErr(hipMalloc(&comm->scratch, scratch), "hipMalloc scratch"));
    NCCLCHECK(hipErr(hipMemset(comm->scratch, 0, scratch), "hipMemset scratch"));
    comm->scratchSize = scratch;
  }
  return ncclSuccess;
}

// What every rank contributes to the split decision (all ranks must reach the same splits).
// It also carries the knobs and the per-algorithm send runs: launch geometry (split, merge,
// ring channels, protocol gates, FIFO sizes) must be identical on every rank, or the two ends of
// a connection would cut different FIFO steps.
struct SplitRecord {
  char host[64];
  char bus[32];
  int32_t nAlgos;
  int32_t nBlocks[kMaxAlgos];
  int32_t sendRun[kMaxAlgos];
  int32_t nFuse[kMaxAlgos];
  int16_t fuse[kMaxAlgos][kMaxFuse][2];  // (channel, peer) of each fusable exchange (fusableTbs)
  uint8_t lowered[kMaxAlgos];             // analyzeLowering found the schedule a one-hop fold (1), with a
                                          // two-phase form (3)
  uint8_t pairShape[kMaxAlgos];           // in pair form when its offered exchanges fuse (pairFormOf)
  uint8_t pairRun[kMaxAlgos];             // pairShape and the pair kernel on
  Knobs knobs;
};

SplitRecord makeSplitRecord(ncclComm* comm) {
  SplitRecord s;
  memset(&s, 0, sizeof(s));
  gethostname(s.host, sizeof(s.host) - 1);
  if (hipDeviceGetPCIBusId(s.bus, sizeof(s.bus) - 1, comm->cudaDev) != hipSuccess)
    snprintf(s.bus, sizeof(s.bus), "dev%d", comm->cudaDev);
  s.nAlgos = (int32_t)comm->algos.size();
  for (size_t a = 0; a < comm->algos.size() && a < (size_t)kMaxAlgos; a++) {
    s.nBlocks[a] = comm->algos[a].nBlocks;
    s.sendRun[a] = algoSendRunOf(comm->algos[a]);
    s.lowered[a] = a < comm->algoFold.size() && !comm->algoFold[a].order.empty()
                       ? (comm->algoFold[a].owner.empty() ? 1 : 3)
                       : 0;
    if (a < comm->algoDirect.size() && comm->algoDirect[a].coll >= 0) s.lowered[a] |= 4;
    const std::vector<FuseCandidate> fc = fusableTbs(comm->algos[a]);
    s.pairShape[a] = comm->knobs.fuse && pairFormOf(comm->algos[a], fc).src >= 0;
    s.pairRun[a] = s.pairShape[a] && comm->knobs.pairKernel;
    for (size_t i = 0; i < fc.size() && s.nFuse[a] < kMaxFuse; i++) {
      s.fuse[a][s.nFuse[a]][0] = fc[i].chan;
      s.fuse[a][s.nFuse[a]][1] = fc[i].peer;
      s.nFuse[a]++;
    }
  }
  s.knobs = comm->knobs;
  s.knobs.smallKernel = 0;  // a rank-local choice: both kernels cut the same FIFO steps
  s.knobs.pairKernel = 0;   // likewise
  return s;
}

// The environment variables behind the Knobs fields in which a and b differ.
static std::string knobDiff(const Knobs& a, const Knobs& b) {
  std::string out;
  auto add = [&](bool differ, const char* name) {
    if (differ) out += std::string(out.empty() ? "" : ", ") + name;
  };
  add(a.mscclOn != b.mscclOn || a.ringOn != b.ringOn || a.treeOn != b.treeOn, "NCCL_ALGO");
  add(memcmp(a.protoOn, b.protoOn, sizeof(a.protoOn)) != 0, "NCCL_PROTO");
  add(a.nthreads != b.nthreads, "NCCL_NTHREADS");
  add(a.ll128Nthreads != b.ll128Nthreads, "NCCL_LL128_NTHREADS");
  add(a.buffSizes[0] != b.buffSizes[0], "NCCL_LL_BUFFSIZE");
  add(a.buffSizes[1] != b.buffSizes[1], "NCCL_LL128_BUFFSIZE");
  add(a.buffSizes[2] != b.buffSizes[2], "NCCL_BUFFSIZE");
  add(a.ringChannels != b.ringChannels, "MSCCL_AMD_RING_CHANNELS");
  add(a.split != b.split, "MSCCL_AMD_SPLIT");
  add(a.targetWgs != b.targetWgs, "MSCCL_AMD_TARGET_WGS");
  add(a.merge != b.merge, "MSCCL_AMD_MERGE");
  add(a.ringFallback != b.ringFallback, "MSCCL_AMD_RING_FALLBACK");
  add(a.ll128Remote != b.ll128Remote, "MSCCL_AMD_LL128_REMOTE");
  add(a.treeMaxBytes != b.treeMaxBytes, "MSCCL_AMD_TREE_MAX_BYTES");
  add(a.smallKernel != b.smallKernel, "MSCCL_AMD_SMALL_KERNEL");
  add(a.referenceSelection != b.referenceSelection, "MSCCL_AMD_REFERENCE_SELECTION");
  add(a.fuse != b.fuse, "MSCCL_AMD_FUSE");
  add(a.treeFlat != b.treeFlat, "MSCCL_AMD_TREE_FLAT");
  add(a.lower != b.lower, "MSCCL_AMD_LOWER");
  add(a.lowerMaxBytes != b.lowerMaxBytes, "MSCCL_AMD_LOWER_MAX_BYTES");
  add(a.lowerLarge != b.lowerLarge, "MSCCL_AMD_LOWER_LARGE");
  add(a.forceRemote != b.forceRemote, "MSCCL_AMD_FORCE_REMOTE");
  add(a.twoPhaseStep != b.twoPhaseStep, "MSCCL_AMD_TWO_PHASE_STEP");
  add(a.direct != b.direct, "MSCCL_AMD_DIRECT");
  return out.empty() ? "(unnamed field)" : out;
}

ncclResult_t applySplits(ncclComm* comm, const std::vector<SplitRecord>& recs) {
  Knobs agreed = comm->knobs;
  agreed.smallKernel = 0;
  agreed.pairKernel = 0;
  for (size_t r = 0; r < recs.size(); r++) {
    if (memcmp(&recs[r].knobs, &agreed, sizeof(Knobs)) != 0) {
      WARN("MSCCL: rank %zu runs with different settings than rank %d: %s (they shape the FIFO steps and must "
           "agree across ranks)", r, comm->rank, knobDiff(recs[r].knobs, agreed).c_str());
      return ncclInvalidUsage;
    }
    if (recs[r].nAlgos != (int32_t)comm->algos.size()) {
      WARN("MSCCL: rank %zu loaded %d MSCCL algorithms, rank %d loaded %zu", r, recs[r].nAlgos, comm->rank,
           comm->algos.size());
      return ncclInvalidUsage;
    }
  }
  int maxCo = 1;
  for (auto& r : recs) {
    int c = 0;
    for (auto& q : recs) c += !strcmp(r.host, q.host) && !strcmp(r.bus, q.bus);
    maxCo = std::max(maxCo, c);
  }
  const SplitRecord& mine = recs[comm->rank];
  comm->coResident = 0;
  for (auto& q : recs) comm->coResident += !strcmp(mine.host, q.host) && !strcmp(mine.bus, q.bus);
  comm->algoSplit.assign(comm->algos.size(), 1);
  comm->algoSplitBase.assign(comm->algos.size(), 1);
  comm->algoMaxBlocks.assign(comm->algos.size(), 1);
  comm->algoSendRun.assign(comm->algos.size(), 1);
  comm->maxSplit = 1;
  for (size_t a = 0; a < comm->algos.size(); a++) {
    int mb = 0, run = 1;
    for (auto& r : recs)
      if ((int)a < r.nAlgos && a < (size_t)kMaxAlgos) {
        mb = std::max(mb, (int)r.nBlocks[a]);
        run = std::max(run, (int)r.sendRun[a]);
      }
    // two ranks sharing a GPU: LL schedules get the wide budget for their large calls
    const bool wide = maxCo == 2 && comm->algos[a].proto == kProtoLL;
    comm->algoSplit[a] = chooseSplit(mb, maxCo, comm->knobs, comm->algos[a].proto, wide);
    comm->algoSplitBase[a] = chooseSplit(mb, maxCo, comm->knobs, comm->algos[a].proto);
    comm->algoMaxBlocks[a] = std::max(1, mb);
    comm->algoSendRun[a] = run;
    comm->maxSplit = std::max(comm->maxSplit, comm->algoSplit[a]);
  }
  // every rank on one GPU: the local Simple FIFO size (plan.h: kLocalSimpleBuff), the same
  // decision on every rank (the same records).  Only when every Simple schedule sends at most
  // two chunks before it receives: a call moves up to chunkSize = half the FIFO per chunk, and a
  // longer run of sends must fit the FIFO whole while its peer sends too (RCCL's 8-rank Simple
  // all-pairs sends 8 chunks first: it keeps the reference's size)
  if (useLocalSimpleFifo(maxCo == (int)recs.size(), comm->knobs, comm->algos, comm->algoSendRun))
    comm->knobs.buffSizes[kProtoSimple] = kLocalSimpleBuff;
  // a schedule runs as the fold only when every rank found it one (the two ends of every flat
  // connection must run the same kernel), and by default not when every rank runs it with the
  // pair kernel: 2 ranks, 128 B - 4 KiB, one instance, graph replay: pair kernel 5.1-5.7 us
  // against the fold's 5.4-6.2 (profiles/r05t_pair_small.txt)
  for (size_t a = 0; a < comm->algoFold.size() && a < (size_t)kMaxAlgos; a++) {
    bool pairEverywhere = comm->knobs.lowerMaxBytes < 0;
    for (auto& r : recs) {
      if ((int)a >= r.nAlgos || !r.lowered[a]) comm->algoFold[a] = ncclComm::FoldProgram();
      pairEverywhere = pairEverywhere && (int)a < r.nAlgos && r.pairRun[a];
    }
    if (pairEverywhere) comm->algoFold[a] = ncclComm::FoldProgram();
    // the two-phase form only where every rank found it (each rank analysed every rank's program)
    for (auto& r : recs)
      if ((int)a >= r.nAlgos || (r.lowered[a] & 2) == 0) comm->algoFold[a].owner.clear();
  }
  // the direct form likewise
  for (size_t a = 0; a < comm->algoDirect.size() && a < (size_t)kMaxAlgos; a++)
    for (auto& r : recs)
      if ((int)a >= r.nAlgos || (r.lowered[a] & 4) == 0) comm->algoDirect[a] = ncclComm::DirectProgram();
  // Lowered large calls (plan.cc: lowerLargePlan): 2 ranks run the pair kernel on the flat
  // connections, more ranks the two-phase fold, each with up to flatSubs workgroups per rank and
  // one flat sub-connection per workgroup: one workgroup per CU over the GPU's co-resident ranks
  // (MSCCL_AMD_TARGET_WGS, default 256), at least kFlatSubs (the fold kernel's).  Agreed: the
  // same records on every rank.
  comm->flatSubs = kFlatSubs;
  if (comm->knobs.lowerLarge) {
    bool any = false;
    for (size_t a = 0; a < comm->algoFold.size(); a++)
      any = any || (!comm->algoFold[a].order.empty() && (recs.size() == 2 || !comm->algoFold[a].owner.empty()));
    if (any) {
      const int target = comm->knobs.targetWgs > 0 ? comm->knobs.targetWgs : 256;
      int w = kFlatSubs;
      while (w * 2 <= kMaxFlatSubs && (int64_t)w * 2 * maxCo <= target) w *= 2;
      comm->flatSubs = w;
    }
  }
  // a schedule in pair form on every rank merges its calls into one pass (enqueue.cc: makeWork);
  // the pass cut decides which workgroup owns which positions, so every rank must agree on it
  comm->algoPairAll.assign(comm->algos.size(), 0);
  for (size_t a = 0; a < comm->algos.size() && a < (size_t)kMaxAlgos; a++) {
    bool all = true;
    for (auto& r : recs) all = all && (int)a < r.nAlgos && r.pairShape[a];
    comm->algoPairAll[a] = all ? 1 : 0;
  }
  // an exchange runs fused only when both ends offered it (fusableTbs)
  comm->algoFuse.assign(comm->algos.size(), {});
  for (size_t a = 0; a < comm->algos.size() && a < (size_t)kMaxAlgos && comm->knobs.fuse; a++) {
    auto offered = [&](int rank, int chan, int peer) {
      const SplitRecord& r = recs[rank];
      if ((int)a >= r.nAlgos) return false;
      for (int i = 0; i < r.nFuse[a]; i++)
        if (r.fuse[a][i][0] == chan && r.fuse[a][i][1] == peer) return true;
      return false;
    };
    for (const FuseCandidate& f : fusableTbs(comm->algos[a]))
      if (f.peer < (int)recs.size() && offered(comm->rank, f.chan, f.peer) && offered(f.peer, f.chan, comm->rank))
        comm->algoFuse[a].push_back(f);
  }
  INFO(kSubInit, "rank %d: %d co-resident ranks per GPU (max), %d sub-connections per connection", comm->rank,
       maxCo, comm->maxSplit);
  return ncclSuccess;
}

// Dependency flags and launch epochs (the reference's mscclFlag array and workIndex,
// init.cc:300-304): every schedule (each loaded algorithm, each ring / tree program, the flat
// fold) owns a range of slots, one per workgroup it can run (thread blocks x maxSplit; the fold:
// kFlatSubs).  A launch reads its epoch from its own slot and advances its own range only
// (interpreter.h: epilogue), so no launch touches another schedule's words.
static ncclResult_t allocSlots(ncclComm* comm) {
  int total = 0;
  auto take = [&](DevAlgoHost& d, int count) {
    d.slotBase = total;
    d.slotCount = count;
    total += count;
  };
  for (DevAlgoHost& d : comm->devAlgos) take(d, std::max(1, d.nBlocks) * comm->maxSplit);
  for (int k = 0; k < 5; k++) take(comm->ringAlgos[k], std::max(1, comm->ringAlgos[k].nBlocks) * comm->maxSplit);
  take(comm->ringAlgos[5], comm->flatSubs);
  for (DevAlgoHost& d : comm->foldAlgos) take(d, comm->flatSubs);  // lowered schedules (lower.cc)
  comm->slotTotal = total;
  const size_t flagWords = (size_t)total * kFlagStride + total;
  NCCLCHECK(hipErr(hipMalloc(&comm->dFlags, flagWords * sizeof(uint64_t)), "hipMalloc flags"));
  NCCLCHECK(hipErr(hipMemset(comm->dFlags, 0, flagWords * sizeof(uint64_t)), "hipMemset"));
  // flags start at 0, the first launch runs epoch 1 (the reference's workIndex, init.cc:300-302)
  const std::vector<uint64_t> epoch0(total, 1);
  NCCLCHECK(hipErr(hipMemcpy(comm->dFlags + (size_t)total * kFlagStride, epoch0.data(), total * sizeof(uint64_t),
                             hipMemcpyHostToDevice), "hipMemcpy epoch"));
  return ncclSuccess;
}

ncclResult_t commFinish(ncclComm* comm) {
  comm->foldClasses.assign(comm->algos.size(), 0);
  comm->foldTwoPhase.assign(comm->algos.size(), 0);
  for (size_t a = 0; a < comm->algoFold.size() && a < comm->algos.size(); a++) {
    comm->foldClasses[a] = (int)comm->algoFold[a].order.size();
    comm->foldTwoPhase[a] = comm->algoFold[a].owner.empty() ? 0 : 1;
  }
  comm->directClasses.assign(comm->algos.size(), 0);
  for (size_t a = 0; a < comm->algoDirect.size() && a < comm->algos.size(); a++)
    if (comm->algoDirect[a].coll >= 0) comm->directClasses[a] = std::max<int>(1, (int)comm->algoDirect[a].order.size());
  PlanContext& pc = comm->planCtx;
  pc.algos = &comm->algos;
  pc.regs = &comm->regs;
  pc.knobs = &comm->knobs;
  pc.foldClasses = &comm->foldClasses;
  pc.foldTwoPhase = &comm->foldTwoPhase;
  pc.directClasses = &comm->directClasses;
  pc.oneLaunch = comm->clique != 0;
  pc.ringDirect = pc.oneLaunch && comm->knobs.direct && lowerOffered();
  pc.flat = flatEnabled(comm);
  pc.ringFallback = comm->ringFallback;
  pc.scratchSize = comm->scratchSize;
  NCCLCHECK(algoUpload(comm));
  NCCLCHECK(allocSlots(comm));
  DevComm dc;
  memset(&dc, 0, sizeof(dc));
  dc.flags = comm->dFlags;
  dc.abortFlag = comm->devAbort;
  dc.errWord = comm->devErr;
  dc.timeoutTicks = comm->timeoutTicks;
  dc.maxSplit = comm->maxSplit;
  dc.llFlagMask = comm->llFlagMask;
  dc.llCleanMask = comm->llCleanMask;
  if (envInt("MSCCL_AMD_TRACE", 0) > 0) {
    comm->traceLight = envInt("MSCCL_AMD_TRACE", 0) == 2;
    comm->traceEvents = (int)std::max<int64_t>(8, std::min<int64_t>(65535, envInt("MSCCL_AMD_TRACE_EVENTS", 256)));
    size_t bytes = (size_t)kMaxTb * comm->maxSplit * comm->traceEvents * sizeof(TraceEvent);
    NCCLCHECK(hipErr(hipMalloc(&comm->dTrace, bytes), "hipMalloc trace"));
    NCCLCHECK(hipErr(hipMemset(comm->dTrace, 0, bytes), "hipMemset trace"));
    dc.trace = comm->dTrace;
    dc.traceEvents = comm->traceEvents;
  }
  NCCLCHECK(npkitSetup(comm));
  dc.epochs = comm->dFlags + (size_t)comm->slotTotal * kFlagStride;
  dc.unused = nullptr;
  NCCLCHECK(hipErr(hipMalloc(&comm->dComm, sizeof(DevComm)), "hipMalloc devComm"));
  NCCLCHECK(hipErr(hipMemcpy(comm->dComm, &dc, sizeof(dc), hipMemcpyHostToDevice), "hipMemcpy"));
  NCCLCHECK(hipErr(hipDeviceSynchronize(), "hipDeviceSynchronize"));
  int nValid = 0;
  for (auto& a : comm->algos) nValid += a.valid;
  if (nValid) INFO(kSubInit, "Connected %d MSCCL algorithms", nValid);  // init.cc:841
  return ncclSuccess;
}

struct RankRecord {
  int32_t pid, dev;
  uint64_t arenaPtr;
  hipIpcMemHandle_t handle;
};

ncclResult_t initRankSync(ncclComm* comm, const ncclUniqueId& id) {
  SocketBootstrap* sb = nullptr;
  NCCLCHECK(SocketBootstrap::connect(id, comm->rank, comm->nRanks, &sb));
  comm->boot = sb;
  comm->ownsBoot = true;
  NCCLCHECK(commLocalSetup(comm));
  const int n = comm->nRanks;
  if (n > 1) {
    SplitRecord srec = makeSplitRecord(comm);
    std::vector<char> sall;
    NCCLCHECK(sb->allgather(&srec, sizeof(srec), &sall));
    std::vector<SplitRecord> recs(n);
    memcpy(recs.data(), sall.data(), sizeof(SplitRecord) * n);
    NCCLCHECK(applySplits(comm, recs));
    NCCLCHECK(transportPlan(comm));
    RankRecord rec;
    memset(&rec, 0, sizeof(rec));
    rec.pid = getpid();
    rec.dev = comm->cudaDev;
    rec.arenaPtr = (uint64_t)comm->arena;
    NCCLCHECK(hipErr(hipIpcGetMemHandle(&rec.handle, comm->arena), "hipIpcGetMemHandle"));
    std::vector<char> all;
    NCCLCHECK(sb->allgather(&rec, sizeof(rec), &all));
    size_t tbytes = comm->table.size() * sizeof(PeerOffsets);
    std::vector<char> tall;
    NCCLCHECK(sb->allgather(comm->table.data(), tbytes, &tall));
    std::vector<std::vector<PeerOffsets>> tables(n);
    comm->peerArena.assign(n, nullptr);
    comm->peerArenaIpc.assign(n, false);
    // a peer is remote (xGMI) unless it runs on the same GPU: same host and PCI bus id
    std::vector<int> peerRemote(n, 0);
    for (int r = 0; r < n; r++) {
      // MSCCL_AMD_FORCE_REMOTE: a test knob (xGMI ordering on one GPU), agreed through the knobs
      // (it changes the lowering limit, plan.cc: defaultLowerMaxBytes)
      peerRemote[r] = strcmp(recs[r].host, srec.host) != 0 || strcmp(recs[r].bus, srec.bus) != 0 ||
                      comm->knobs.forceRemote != 0;
      if (r != comm->rank && peerRemote[r]) comm->anyRemote = true;
    }
    for (int r = 0; r < n; r++) {
      tables[r].resize(comm->table.size());
      memcpy(tables[r].data(), tall.data() + (size_t)r * tbytes, tbytes);
      RankRecord pr;
      memcpy(&pr, all.data() + (size_t)r * sizeof(RankRecord), sizeof(pr));
      if (r == comm->rank) {
        comm->peerArena[r] = comm->arena;
      } else if (pr.pid == rec.pid) {
        if (pr.dev != comm->cudaDev) {
          hipError_t e = hipDeviceEnablePeerAccess(pr.dev, 0);
          if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return hipErr(e, "hipDeviceEnablePeerAccess");
          (void)hipGetLastError();
        }
        comm->peerArena[r] = (char*)pr.arenaPtr;
      } else {
        void* p = nullptr;
        NCCLCHECK(hipErr(hipIpcOpenMemHandle(&p, pr.handle, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle"));
        comm->peerArena[r] = (char*)p;
        comm->peerArenaIpc[r] = true;
      }
    }
    NCCLCHECK(transportConnect(comm, tables, comm->peerArena, peerRemote));
  }
  NCCLCHECK(commFinish(comm));
  NCCLCHECK(sb->barrier());
  return ncclSuccess;
}

}  // namespace

ncclResult_t commFree(ncclComm* comm, bool peerBarrier) {
  if (!comm) return ncclSuccess;
  hipSetDevice(comm->cudaDev);
  hipDeviceSynchronize();
  for (auto& d : comm->devAlgos) {
    if (d.dImages) hipFree(d.dImages);
    if (d.dSend) hipFree(d.dSend);
    if (d.dRecv) hipFree(d.dRecv);
  }
  for (auto& d : comm->ringAlgos)
    if (d.dImages) hipFree(d.dImages);  // their connection records are comm->ringSend / ringRecv
  for (auto& d : comm->foldAlgos)
    if (d.dImages) hipFree(d.dImages);  // the flat connections (comm->flatSend / flatRecv)
  for (auto& d : comm->directAlgos)
    if (d.dImages) hipFree(d.dImages);  // no connections
  if (comm->ringDirectRS.dImages) hipFree(comm->ringDirectRS.dImages);
  if (comm->ringSend) hipFree(comm->ringSend);
  if (comm->ringRecv) hipFree(comm->ringRecv);
  if (comm->treeSend) hipFree(comm->treeSend);
  if (comm->treeRecv) hipFree(comm->treeRecv);
  if (comm->flatSend) hipFree(comm->flatSend);
  if (comm->flatRecv) hipFree(comm->flatRecv);
  for (size_t r = 0; r < comm->peerArena.size(); r++)
    if (comm->peerArenaIpc[r] && comm->peerArena[r]) hipIpcCloseMemHandle(comm->peerArena[r]);
  if (comm->dComm) hipFree(comm->dComm);
  if (comm->dFlags) hipFree(comm->dFlags);
  if (comm->dTrace) hipFree(comm->dTrace);
  if (comm->dNpkit && comm->dComm) npkitDump(comm, nullptr);  // NPKIT_TEARDOWN (npkit.h:214-219)
  npkitFree(comm);
  if (comm->scratch) hipFree(comm->scratch);
  if (comm->boot && comm->ownsBoot) {
    if (peerBarrier) comm->boot->barrier();  // peers may still read our arena until everyone is done
    delete comm->boot;
  }
  if (comm->arena) hipFree(comm->arena);
  if (comm->hostAbort) hipHostFree(comm->hostAbort);
  if (comm->hostErr) hipHostFree(comm->hostErr);
  if (comm->doneEvent) hipEventDestroy(comm->doneEvent);
  comm->magic = 0;  // commPoison (init.cc:108-110)
  delete comm;
  return ncclSuccess;
}

}  // namespace msccl

extern "C" {

ncclResult_t ncclGetVersion(int* version) {
  if (!version) return ncclInvalidArgument;
  *version = NCCL_VERSION_CODE;
  return ncclSuccess;
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* out) {
  initEnv();  // ncclInit -> initEnv (init.cc:70-85, misc/param.cc:51-60)
  if (!out) { WARN("ncclGetUniqueId : uniqueId argument is NULL"); return ncclInvalidArgument; }
  return bootstrapCreateRoot(out);
}

ncclResult_t ncclCommInitRank(ncclComm_t* newcomm, int nranks, ncclUniqueId commId, int myrank) {
  initEnv();
  if (!newcomm) { WARN("ncclCommInitRank : comm argument is NULL"); return ncclInvalidArgument; }
  if (nranks < 1 || myrank < 0 || myrank >= nranks) {
    WARN("Invalid rank requested : %d/%d", myrank, nranks);
    return ncclInvalidArgument;
  }
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return ncclUnhandledCudaError;
  ncclComm* comm = new ncclComm();
  comm->rank = myrank;
  comm->nRanks = nranks;
  comm->cudaDev = dev;
  *newcomm = comm;
  if (groupActive()) {
    // ncclGroupStart/End around InitRank: run all inits in parallel at group end (group.cc:165-187)
    groupAddInit([comm, commId]() { return initRankSync(comm, commId); }, comm);
    return ncclSuccess;
  }
  ncclResult_t r = initRankSync(comm, commId);
  if (r != ncclSuccess) {
    commFree(comm, false);
    *newcomm = nullptr;
  }
  return r;
}

// Single process, ndev ranks (init.cc:1099-1117).  devlist may repeat a device: such ranks are
// co-resident on one GPU and a group of their calls becomes one fused launch.
ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int* devlist) {
  initEnv();
  if (!comms) { WARN("ncclCommInitAll : comms argument is NULL"); return ncclInvalidArgument; }
  if (ndev < 1) { WARN("ncclCommInitAll : invalid ndev %d", ndev); return ncclInvalidArgument; }
  int ndevices = 0;
  if (hipGetDeviceCount(&ndevices) != hipSuccess) return ncclUnhandledCudaError;
  int saved = 0;
  hipGetDevice(&saved);
  {
    // a group of co-resident ranks runs as ONE launch whose workgroups spin on each other;
    // kMaxLaunchRanks bounds the ranks one launch carries (enqueue.cc: launchGroup)
    std::vector<int> perDev(std::max(ndevices, 1), 0);
    for (int i = 0; i < ndev; i++) {
      int dev = devlist ? devlist[i] : i;
      if (dev >= 0 && dev < ndevices && ++perDev[dev] > kMaxLaunchRanks) {
        WARN("ncclCommInitAll : more than %d ranks on device %d; co-resident ranks run in one launch and at most %d "
             "fit", kMaxLaunchRanks, dev, kMaxLaunchRanks);
        return ncclInvalidUsage;
      }
    }
  }
  std::vector<ncclComm*> cs(ndev);
  ncclResult_t res = ncclSuccess;
  // every rank on one device: one clique, whose group calls are one fused launch (comm.h: clique)
  bool oneDevice = ndev > 1;
  for (int i = 1; i < ndev && oneDevice; i++) oneDevice = (devlist ? devlist[i] : i) == (devlist ? devlist[0] : 0);
  static std::atomic<uint64_t> cliques{0};
  const uint64_t clique = oneDevice ? ++cliques : 0;
  for (int i = 0; i < ndev && res == ncclSuccess; i++) {
    int dev = devlist ? devlist[i] : i;
    if (dev < 0 || dev >= ndevices) {
      WARN("ncclCommInitAll : invalid device %d", dev);
      res = ncclInvalidArgument;
      break;
    }
    ncclComm* c = new ncclComm();
    c->rank = i;
    c->nRanks = ndev;
    c->cudaDev = dev;
    c->clique = clique;
    cs[i] = c;
    res = commLocalSetup(c);
  }
  if (res == ncclSuccess && ndev > 1) {
    std::vector<SplitRecord> recs(ndev);
    for (int i = 0; i < ndev; i++) recs[i] = makeSplitRecord(cs[i]);
    for (int i = 0; i < ndev && res == ncclSuccess; i++) {
      res = applySplits(cs[i], recs);
      if (res != ncclSuccess) break;
      hipSetDevice(cs[i]->cudaDev);
      res = transportPlan(cs[i]);
    }
  }
  if (res == ncclSuccess && ndev > 1) {
    std::vector<std::vector<PeerOffsets>> tables(ndev);
    std::vector<char*> bases(ndev);
    for (int i = 0; i < ndev; i++) {
      tables[i] = cs[i]->table;
      bases[i] = cs[i]->arena;
    }
    for (int i = 0; i < ndev && res == ncclSuccess; i++) {
      hipSetDevice(cs[i]->cudaDev);
      for (int j = 0; j < ndev; j++) {
        if (cs[j]->cudaDev != cs[i]->cudaDev) {
          hipError_t e = hipDeviceEnablePeerAccess(cs[j]->cudaDev, 0);
          if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
            WARN("hipDeviceEnablePeerAccess(%d -> %d) failed: %s", cs[i]->cudaDev, cs[j]->cudaDev, hipGetErrorString(e));
            res = ncclUnhandledCudaError;
          }
          (void)hipGetLastError();
        }
      }
      std::vector<int> remote(ndev);
      for (int j = 0; j < ndev; j++) {
        remote[j] = cs[j]->cudaDev != cs[i]->cudaDev || cs[i]->knobs.forceRemote != 0;
        if (j != i && remote[j]) cs[i]->anyRemote = true;
      }
      cs[i]->peerArena = bases;
      cs[i]->peerArenaIpc.assign(ndev, false);
      if (res == ncclSuccess) res = transportConnect(cs[i], tables, bases, remote);
    }
  }
  for (int i = 0; i < ndev && res == ncclSuccess; i++) {
    hipSetDevice(cs[i]->cudaDev);
    res = commFinish(cs[i]);
  }
  hipSetDevice(saved);
  if (res != ncclSuccess) {
    for (auto* c : cs)
      if (c) commFree(c, false);
    return res;
  }
  for (int i = 0; i < ndev; i++) comms[i] = cs[i];
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  if (comm == nullptr) return ncclSuccess;
  if (!commValid(comm)) { WARN("comm %p has already been destroyed", (void*)comm); return ncclInvalidArgument; }
  int saved = 0;
  hipGetDevice(&saved);
  ncclResult_t r = commFree(comm, true);
  hipSetDevice(saved);
  return r;
}

ncclResult_t ncclCommAbort(ncclComm_t comm) {
  if (comm == nullptr) return ncclSuccess;
  if (!commValid(comm)) return ncclInvalidArgument;
  __atomic_store_n(comm->hostAbort, 1u, __ATOMIC_SEQ_CST);  // kernels poll it in every spin (init.cc:1197)
  int saved = 0;
  hipGetDevice(&saved);
  ncclResult_t r = commFree(comm, false);
  hipSetDevice(saved);
  return r;
}

const char* ncclGetErrorString(ncclResult_t code) {
  switch (code) {
    case ncclSuccess: return "no error";
    case ncclUnhandledCudaError: return "unhandled cuda error";
    case ncclSystemError: return "unhandled system error";
    case ncclInternalError: return "internal error";
    case ncclInvalidArgument: return "invalid argument";
    case ncclInvalidUsage: return "invalid usage";
    default: return "unknown result code";
  }
}

ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* asyncError) {
  if (!commValid(comm) || !asyncError) return ncclInvalidArgument;
  uint32_t e = __atomic_load_n(comm->hostErr, __ATOMIC_SEQ_CST);
  if (e == kDevTimeout) comm->asyncError = ncclSystemError;
  else if (e == kDevAbort) comm->asyncError = ncclSystemError;
  else if (e != 0) comm->asyncError = ncclInternalError;
  *asyncError = comm->asyncError;
  return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
  if (!commValid(comm) || !count) return ncclInvalidArgument;
  *count = comm->nRanks;
  return ncclSuccess;
}

ncclResult_t ncclCommCuDevice(const ncclComm_t comm, int* devid) {
  if (!commValid(comm) || !devid) return ncclInvalidArgument;
  *devid = comm->cudaDev;
  return ncclSuccess;
}

ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank) {
  if (!commValid(comm) || !rank) return ncclInvalidArgument;
  *rank = comm->rank;
  return ncclSuccess;
}

const char* ncclGetLastError(ncclComm_t comm) { return lastError(); }



}  // extern "C"

// Introspection C-ABI (include/msccl_amd.h).
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <sstream>

#include <hip/hip_runtime.h>

#include "../../include/msccl_amd.h"
#include "algo.h"
#include "bootstrap.h"
#include "comm.h"
#include "debug.h"
#include "lower.h"
#include "plan.h"

using namespace msccl;

static int putOut(const std::string& s, char* out, size_t len) {
  if (!out || len == 0) return ncclInvalidArgument;
  if (s.size() + 1 > len) return ncclInvalidArgument;
  memcpy(out, s.c_str(), s.size() + 1);
  return 0;
}

extern "C" {

int mscclAmdAlgoJson(const char* xmlPath, int rank, int nranks, char* out, size_t outLen) {
  Algorithm a;
  int r = loadAlgoFromXml(xmlPath, &a, kMaxChannels, rank, nranks);
  if (r != 0) return r;
  return putOut(algoToJson(a), out, outLen);
}

int mscclAmdFusableJson(const char* xmlPath, int rank, int nranks, char* out, size_t outLen) {
  Algorithm a;
  int r = loadAlgoFromXml(xmlPath, &a, kMaxChannels, rank, nranks);
  if (r != 0) return r;
  std::ostringstream o;
  o << "{\"fusable\":[";
  const std::vector<FuseCandidate> fc = fusableTbs(a);
  for (size_t i = 0; i < fc.size(); i++)
    o << (i ? "," : "") << "[" << fc[i].tb << "," << fc[i].index << "," << fc[i].chan << "," << fc[i].peer << "]";
  o << "],\"sendcopy\":[";
  bool first = true;
  for (int b = 0; b < a.nBlocks; b++)
    for (size_t i = 0; i + 1 < a.tbs[b].transfers.size(); i++)
      if (sendCopyFusable(a, a.tbs[b].transfers, i)) {
        o << (first ? "" : ",") << "[" << b << "," << i << "]";
        first = false;
      }
  o << "]}";
  return putOut(o.str(), out, outLen);
}

int mscclAmdLowerJson(const char* xmlPath, int nranks, char* out, size_t outLen) {
  if (!xmlPath || nranks < 1) return ncclInvalidArgument;
  std::vector<Algorithm> byRank(nranks);
  for (int r = 0; r < nranks; r++) {
    const int res = loadAlgoFromXml(xmlPath, &byRank[r], kMaxChannels, r, nranks);
    if (res != 0) return res;
  }
  const FoldLowering fl = analyzeFoldLowering(byRank);
  std::ostringstream o;
  o << "{\"ok\":" << (fl.ok ? 1 : 0);
  if (fl.ok) {
    // "classes": per class of chunks, every rank's fold order; "chunkClass": every chunk's class
    o << ",\"classes\":[";
    for (size_t k = 0; k < fl.order.size(); k++) {
      o << (k ? "," : "") << "[";
      for (size_t r = 0; r < fl.order[k].size(); r++) {
        o << (r ? "," : "") << "[";
        for (size_t i = 0; i < fl.order[k][r].size(); i++) o << (i ? "," : "") << fl.order[k][r][i];
        o << "]";
      }
      o << "]";
    }
    o << "],\"chunkClass\":[";
    for (size_t c = 0; c < fl.chunkClass.size(); c++) o << (c ? "," : "") << fl.chunkClass[c];
    // the two-phase form: every chunk's owner (lower.h), or why there is none
    o << "],\"twoPhase\":" << (fl.twoPhase ? 1 : 0);
    if (fl.twoPhase) {
      o << ",\"owner\":[";
      for (size_t c = 0; c < fl.owner.size(); c++) o << (c ? "," : "") << fl.owner[c];
      o << "]";
    } else {
      o << ",\"whyNotTwoPhase\":\"" << fl.whyNotTwoPhase << "\"";
    }
  } else {
    o << ",\"why\":\"" << fl.why << "\"";
  }
  o << "}";
  return putOut(o.str(), out, outLen);
}

int mscclAmdDirectJson(const char* xmlPath, int nranks, char* out, size_t outLen) {
  if (!xmlPath || nranks < 1) return ncclInvalidArgument;
  std::vector<Algorithm> byRank(nranks);
  for (int r = 0; r < nranks; r++) {
    const int res = loadAlgoFromXml(xmlPath, &byRank[r], kMaxChannels, r, nranks);
    if (res != 0) return res;
  }
  const DirectLowering dl = analyzeDirectLowering(byRank);
  std::ostringstream o;
  o << "{\"ok\":" << (dl.ok ? 1 : 0) << ",\"coll\":" << dl.coll;
  if (dl.ok) {
    o << ",\"classes\":[";
    for (size_t k = 0; k < dl.order.size(); k++) {
      o << (k ? "," : "") << "[";
      for (size_t r = 0; r < dl.order[k].size(); r++) {
        o << (r ? "," : "") << "[";
        for (size_t i = 0; i < dl.order[k][r].size(); i++) o << (i ? "," : "") << dl.order[k][r][i];
        o << "]";
      }
      o << "]";
    }
    o << "],\"chunkClass\":[";
    for (size_t c = 0; c < dl.chunkClass.size(); c++) o << (c ? "," : "") << dl.chunkClass[c];
    o << "]";
  } else {
    o << ",\"why\":\"" << dl.why << "\"";
  }
  o << "}";
  return putOut(o.str(), out, outLen);
}

// the collective the fold kernel would run for this fallback plan (plan.cc: makeFlatTreePlan;
// kRingAllReduce / kRingReduceScatter / kRingAllGather), 0 when the call keeps the ring / chain
static int flatOf(const CallDesc& c, const Knobs& k, Plan rp) {
  return makeFlatTreePlan(c, k, &rp) == 0 ? rp.flatColl : 0;
}

int mscclAmdPlanJson(const char* xmlFiles, int rank, int nranks, int coll, size_t count, int dtype, int redop,
                     int inPlace, char* out, size_t outLen) {
  std::vector<Algorithm> algos;
  loadAlgosFromXmlFiles(xmlFiles, &algos, kMaxChannels, rank, nranks);
  CallDesc c;
  c.coll = coll;
  c.count = count;
  c.dtype = dtype;
  c.redop = redop;
  c.nRanks = nranks;
  c.rank = rank;
  c.inPlace = inPlace != 0;
  std::vector<Registration> regs;
  const Knobs k = Knobs::fromEnv();
  int idx = selectAlgo(algos, regs, c, k);
  std::ostringstream o;
  if (idx < 0) {
    o << "{\"algo\":-1,\"nalgos\":" << algos.size();
    Plan rp;
    if (k.ringFallback && nranks > 1 && makeRingPlan(c, k, &rp) == 0)
      o << ",\"ring\":{\"coll\":" << rp.ringColl << ",\"proto\":" << rp.proto << ",\"channels\":" << rp.ringChannels
        << ",\"nthreads\":" << rp.refNthreads << ",\"size\":" << rp.count << ",\"dtype\":" << rp.dtype
        << ",\"nBytes\":" << rp.nBytes << ",\"chunk\":" << rp.chunkSize << ",\"minChunk\":" << rp.minChunk
        << ",\"lastChunk\":" << rp.ringLastChunk << ",\"flat\":" << flatOf(c, k, rp) << "}";
    o << "}";
    return putOut(o.str(), out, outLen);
  }
  Plan p;
  int r = makePlan(algos, idx, -1, c, k, &p);
  if (r != 0) return r;
  o << "{\"algo\":" << idx << ",\"nalgos\":" << algos.size() << ",\"proto\":" << p.proto
    << ",\"nthreads\":" << p.refNthreads << ",\"count\":" << p.count << ",\"dtype\":" << p.dtype
    << ",\"sizeMultiplier\":" << p.sizeMultiplier << ",\"nBytes\":" << p.nBytes
    << ",\"maxAllowedCount\":" << p.maxAllowedCount << ",\"ncpl\":" << p.nchunksPerLoop
    << ",\"sizePerChunk\":" << p.sizePerChunk << ",\"chunkSize\":" << p.chunkSize << ",\"minChunk\":" << p.minChunk
    << ",\"scratchNeeded\":" << p.scratchNeeded << ",\"nIters\":" << p.nIters << "}";
  return putOut(o.str(), out, outLen);
}

int mscclAmdLaunchPlanJson(const char* xmlFiles, int rank, int nranks, int oneGpu, int coll, size_t count, int dtype,
                           int redop, int inPlace, char* out, size_t outLen) {
  if (rank < 0 || nranks < 2 || rank >= nranks) return ncclInvalidArgument;
  // init's decisions for a communicator of nranks ranks, all on one GPU (oneGpu) or spread over
  // several (every rank then has a peer on another GPU): the schedules as this rank loads them,
  // the knobs, the one-hop lowering (lower.cc, on every rank's load; offered only where every
  // rank offers it, which the same environment does), the Simple FIFO size (applySplits)
  std::vector<Algorithm> algos;
  if (xmlFiles) loadAlgosFromXmlFiles(xmlFiles, &algos, kMaxChannels, rank, nranks);
  Knobs k = Knobs::fromEnv();
  const bool flat = k.ringFallback && k.treeFlat && nranks <= kMaxReduceFusion;
  std::vector<int> classes(algos.size(), 0), sendRun(algos.size(), 1), pairAll(algos.size(), 0),
      twoPhase(algos.size(), 0);
  for (size_t a = 0; a < algos.size(); a++) {
    for (int r = 0; r < nranks; r++) {
      Algorithm ar;
      if (loadAlgoFromXml(algos[a].path.c_str(), &ar, kMaxChannels, r, nranks) == 0)
        sendRun[a] = std::max(sendRun[a], algoSendRunOf(ar));
    }
    const Algorithm& g = algos[a];
    // init.cc: applySplits's pair shape, on every rank (the one-pass merge and the pair kernel)
    bool shape = k.fuse && !g.path.empty() && g.ngpus == nranks;
    for (int r = 0; r < nranks && shape; r++) {
      Algorithm ar;
      shape = loadAlgoFromXml(g.path.c_str(), &ar, kMaxChannels, r, nranks) == 0 && pairFormOf(ar, fusableTbs(ar)).src >= 0;
    }
    pairAll[a] = shape ? 1 : 0;
    if (k.lower && flat && lowerOffered() && g.valid && g.coll == kAllReduce && g.proto == kProtoLL && !g.path.empty() &&
        g.ngpus == nranks) {
      const FoldLowering fl = lowerScheduleFile(g.path, nranks);
      if (fl.ok) classes[a] = (int)fl.order.size();
      if (fl.ok && fl.twoPhase) twoPhase[a] = 1;
      // init.cc: applySplits keeps a schedule every rank runs with the pair kernel off the fold
      bool pairEverywhere = k.lowerMaxBytes < 0 && k.fuse && k.pairKernel;
      for (int r = 0; r < nranks && pairEverywhere; r++) {
        Algorithm ar;
        pairEverywhere = loadAlgoFromXml(g.path.c_str(), &ar, kMaxChannels, r, nranks) == 0 &&
                         pairFormOf(ar, fusableTbs(ar)).src >= 0;
      }
      if (pairEverywhere) classes[a] = 0;
    }
  }
  if (useLocalSimpleFifo(oneGpu != 0, k, algos, sendRun)) k.buffSizes[kProtoSimple] = kLocalSimpleBuff;
  std::vector<Registration> regs;
  PlanContext pc;
  pc.algos = &algos;
  pc.regs = &regs;
  pc.knobs = &k;
  pc.foldClasses = &classes;
  pc.foldTwoPhase = &twoPhase;
  pc.flat = flat;
  pc.ringFallback = k.ringFallback != 0;
  pc.scratchSize = (size_t)-1;  // uncapped (MSCCL_AMD_MAX_SCRATCH is not modelled here)
  CallDesc c;
  c.coll = coll;
  c.count = count;
  c.dtype = dtype;
  c.redop = redop;
  c.nRanks = nranks;
  c.rank = rank;
  c.inPlace = inPlace != 0;
  c.remote = oneGpu == 0;
  Plan p;
  const int res = planCall(pc, c, false, &p);
  if (res != 0) return res;
  // an MSCCL call of a schedule in pair form on every rank runs the pair kernel on LL when it is one
  // pass and the knob is on (enqueue.cc: makeWork merges a pair-form call's iterations while a
  // workgroup's sends fit the FIFO: 64 iterations at the default LL FIFO and split 8, the bound
  // used here).  That bound is approximate for a multi-iteration call under a non-default
  // NCCL_LL_BUFFSIZE or a forced MSCCL_AMD_SPLIT (the communicator's merge follows its agreed split
  // and FIFO geometry): "kernelExact" is 0 for those answers.
  const bool pairCall = p.ringColl == 0 && p.algoIndex >= 0 && (size_t)p.algoIndex < pairAll.size() &&
                        pairAll[p.algoIndex] && p.proto == kProtoLL && k.pairKernel && k.smallKernel &&
                        (p.nIters <= 1 || (p.nIters <= 64 && p.sizePerChunk % std::max<int64_t>(1, p.chunkSize) == 0));
  const bool pairMaybe = p.ringColl == 0 && p.algoIndex >= 0 && (size_t)p.algoIndex < pairAll.size() &&
                         pairAll[p.algoIndex] && p.proto == kProtoLL && p.nIters > 1;
  const bool exact = !(pairMaybe && (k.buffSizes[kProtoLL] != (int64_t)8 * 512 * kFifoSteps * 16 || k.split > 0));
  const char* kernel = p.ringColl == kTreeFlat ? (p.lowerMode == kLowerPair       ? "pair"
                                                  : p.lowerMode == kLowerTwoPhase ? "twophase"
                                                                                  : "fold")
                       : p.ringColl == kTreeAllReduce ? "tree" : p.ringColl ? "ring" : pairCall ? "pair" : "interpreter";
  std::ostringstream o;
  o << "{\"kernel\":\"" << kernel << "\",\"kernelExact\":" << (exact ? 1 : 0) << ",\"algo\":" << p.algoIndex
    << ",\"proto\":" << p.proto
    << ",\"lowered\":" << (p.ringColl == kTreeFlat && p.algoIndex >= 0 ? 1 : 0) << ",\"nBytes\":" << p.nBytes
    << ",\"lowerMaxBytes\":" << (k.lowerMaxBytes >= 0 ? k.lowerMaxBytes : defaultLowerMaxBytes(nranks, c.remote))
    << ",\"simpleBuffBytes\":" << k.buffSizes[kProtoSimple] << ",\"remote\":" << (c.remote ? 1 : 0)
    << ",\"pairForm\":" << (p.algoIndex >= 0 && (size_t)p.algoIndex < pairAll.size() ? pairAll[p.algoIndex] : 0)
    << ",\"classes\":[";
  for (size_t a = 0; a < classes.size(); a++) o << (a ? "," : "") << classes[a];
  o << "]}";
  return putOut(o.str(), out, outLen);
}

int mscclAmdCommInfo(ncclComm_t comm, char* out, size_t outLen) {
  if (!commValid(comm)) return ncclInvalidArgument;
  std::ostringstream o;
  o << "{\"rank\":" << comm->rank << ",\"nranks\":" << comm->nRanks << ",\"device\":" << comm->cudaDev
    << ",\"algos\":[";
  for (size_t i = 0; i < comm->algos.size(); i++) {
    const Algorithm& a = comm->algos[i];
    o << (i ? "," : "") << "{\"name\":\"" << a.name << "\",\"proto\":" << a.proto << ",\"coll\":" << a.coll
      << ",\"nBlocks\":" << a.nBlocks << ",\"ncpl\":" << a.nchunksPerLoop << ",\"inplace\":" << a.inPlace
      << ",\"minBytes\":" << a.minBytes << ",\"maxBytes\":" << a.maxBytes << ",\"path\":\"" << a.path << "\"}";
  }
  o << "],\"sendConns\":" << comm->sendKeys.size() << ",\"recvConns\":" << comm->recvKeys.size()
    << ",\"arenaBytes\":" << comm->arenaSize << ",\"scratchBytes\":" << comm->scratchSize
    << ",\"llSlotLines\":" << comm->llSlotLines << ",\"simpleSlotBytes\":" << comm->simpleSlotBytes
    << ",\"workIndex\":" << comm->workIndex << ",\"maxSplit\":" << comm->maxSplit
    << ",\"coResident\":" << comm->coResident << ",\"anyRemote\":" << (comm->anyRemote ? 1 : 0)
    << ",\"algoSplit\":[";
  for (size_t i = 0; i < comm->algoSplit.size(); i++) o << (i ? "," : "") << comm->algoSplit[i];
  o << "],\"algoSendRun\":[";
  for (size_t i = 0; i < comm->algoSendRun.size(); i++) o << (i ? "," : "") << comm->algoSendRun[i];
  o << "],\"algoFuse\":[";  // per algorithm: thread blocks whose s + rrc exchange runs fused
  for (size_t i = 0; i < comm->algoFuse.size(); i++) {
    o << (i ? "," : "") << "[";
    for (size_t j = 0; j < comm->algoFuse[i].size(); j++) o << (j ? "," : "") << comm->algoFuse[i][j].tb;
    o << "]";
  }
  const auto& L = comm->last;
  o << "],\"last\":{\"algo\":" << L.algo << ",\"proto\":" << L.proto << ",\"split\":" << L.split
    << ",\"merge\":" << L.merge << ",\"ringColl\":" << L.ringColl << ",\"ringChannels\":" << L.ringChannels
    << ",\"blocks\":" << L.blocks << ",\"small\":" << L.small << ",\"set\":" << L.set << ",\"pair\":" << L.pair
    << ",\"kernel\":" << L.kernel << "},\"flatSubs\":" << comm->flatSubs << "}";
  return putOut(o.str(), out, outLen);
}

int mscclAmdBootstrapAllgather(const ncclUniqueId* id, int rank, int nranks, const void* mine, size_t bytes,
                               void* out) {
  if (!id) return ncclInvalidArgument;
  SocketBootstrap* b = nullptr;
  ncclResult_t r = SocketBootstrap::connect(*id, rank, nranks, &b);
  if (r != ncclSuccess) return r;
  std::vector<char> all;
  r = b->allgather(mine, bytes, &all);
  if (r == ncclSuccess) memcpy(out, all.data(), all.size());
  delete b;
  return r;
}

int mscclAmdSetEnvFile(const char* path) {
  if (path == nullptr) return ncclInvalidArgument;
  return setEnvFile(path) ? ncclSuccess : ncclSystemError;
}

const char* mscclAmdKernelLayoutMismatch(void) { return kernelLayoutMismatch(); }

int mscclAmdAlgoBlocks(ncclComm_t comm, int algoIndex) {
  if (!commValid(comm) || algoIndex < 0 || algoIndex >= (int)comm->algos.size()) return -1;
  return comm->algos[algoIndex].nBlocks;
}

int mscclAmdTraceRead(ncclComm_t comm, void* out, size_t outBytes, int* slots, int* events) {
  if (!commValid(comm)) return ncclInvalidArgument;
  if (!comm->dTrace) return ncclInvalidUsage;
  const int nSlots = kMaxTb * comm->maxSplit;
  const size_t bytes = (size_t)nSlots * comm->traceEvents * sizeof(TraceEvent);
  if (slots) *slots = nSlots;
  if (events) *events = comm->traceEvents;
  if (!out) return ncclSuccess;
  if (outBytes < bytes) return ncclInvalidArgument;
  if (hipSetDevice(comm->cudaDev) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(out, comm->dTrace, bytes, hipMemcpyDeviceToHost) != hipSuccess)
    return ncclUnhandledCudaError;
  return ncclSuccess;
}

int mscclAmdLineTearProbe(int writerDev, int readerDev, int nLines, int iters, double seconds,
                          unsigned long long* out) {
  if (!out || nLines <= 0 || iters <= 0 || seconds <= 0) return ncclInvalidArgument;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) return ncclUnhandledCudaError;
  if (writerDev < 0 || readerDev < 0 || writerDev >= ndev || readerDev >= ndev) return ncclInvalidArgument;
  int prev = 0;
  (void)hipGetDevice(&prev);
  void* lines = nullptr;
  unsigned long long* cnt = nullptr;
  hipStream_t rs = nullptr, ws = nullptr;
  ncclResult_t res = ncclUnhandledCudaError;
  const size_t bytes = (size_t)nLines * 16;
  do {
    // the receiving device owns the lines, in the uncached memory the FIFOs use (transport.cc)
    if (hipSetDevice(readerDev) != hipSuccess) break;
    if (hipExtMallocWithFlags(&lines, bytes, hipDeviceMallocUncached) != hipSuccess) break;
    if (hipMalloc((void**)&cnt, 3 * sizeof(unsigned long long)) != hipSuccess) break;
    if (hipMemset(lines, 0, bytes) != hipSuccess || hipMemset(cnt, 0, 3 * sizeof(unsigned long long)) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess)
      break;
    if (hipStreamCreateWithFlags(&rs, hipStreamNonBlocking) != hipSuccess) break;
    if (hipSetDevice(writerDev) != hipSuccess) break;
    if (writerDev != readerDev) {
      hipError_t e = hipDeviceEnablePeerAccess(readerDev, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) break;
      (void)hipGetLastError();
    }
    if (hipStreamCreateWithFlags(&ws, hipStreamNonBlocking) != hipSuccess) break;
    // readers first (they bound themselves by time), then the writers
    if (hipSetDevice(readerDev) != hipSuccess) break;
    const int rblocks = std::min(1024, (nLines + 255) / 256);
    if (launchLineReader(lines, nLines, iters, (uint64_t)(seconds * 1e8), cnt, rblocks, rs) != 0) break;
    if (hipSetDevice(writerDev) != hipSuccess) break;
    if (launchLineWriter(lines, nLines, iters, std::min(1024, (nLines + 255) / 256), ws) != 0) break;
    if (hipStreamSynchronize(ws) != hipSuccess) break;
    if (hipSetDevice(readerDev) != hipSuccess || hipStreamSynchronize(rs) != hipSuccess) break;
    if (hipMemcpy(out, cnt, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) break;
    res = ncclSuccess;
  } while (false);
  if (ws) {
    (void)hipSetDevice(writerDev);
    (void)hipStreamDestroy(ws);
  }
  (void)hipSetDevice(readerDev);
  if (rs) (void)hipStreamDestroy(rs);
  if (lines) (void)hipFree(lines);
  if (cnt) (void)hipFree(cnt);
  (void)hipSetDevice(prev);
  return res;
}

}  // extern "C"

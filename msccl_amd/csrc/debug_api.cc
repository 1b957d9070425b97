// Introspection C-ABI (include/msccl_amd.h).
#include <stdio.h>
#include <string.h>

#include <sstream>

#include <hip/hip_runtime.h>

#include "../../include/msccl_amd.h"
#include "algo.h"
#include "bootstrap.h"
#include "comm.h"
#include "debug.h"
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
  o << "]}";
  return putOut(o.str(), out, outLen);
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
        << ",\"lastChunk\":" << rp.ringLastChunk << "}";
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
    << ",\"blocks\":" << L.blocks << ",\"small\":" << L.small << "}}";
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

}  // extern "C"

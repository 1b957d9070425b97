// Collective entry points, group handling and kernel launch.
//
// Replaces the reference's host path for the MSCCL algorithm:
//   collectives/all_reduce.cc:11-19, reduce_scatter.cc:12-20, all_gather.cc:12-20,
//   all_to_all.cc, custom_collective.cc  ->  enqueue
//   ncclEnqueueCheck (enqueue.cc:1456-1527), ncclSetupCollKernel (809-866), computeColl
//   (591-734), ncclLaunchKernel (337-378), nRanks==1 memcpy path (811-816), workIndex/flag
//   reset (714-721), group.cc:95-408.
// One fused launch per (device, kernel variant) and group round: a rank's thread blocks
// occupy blocks [blockBase, blockBase + nBlocks) of the grid.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <thread>
#include <tuple>
#include <vector>

#include "comm.h"
#include "debug.h"
#include "group.h"
#include "plan.h"

namespace msccl {

namespace {
thread_local int tGroupDepth = 0;
thread_local std::vector<CollOp> tOps;
thread_local std::vector<std::pair<std::function<ncclResult_t()>, ncclComm*>> tInits;
thread_local ncclResult_t tGroupError = ncclSuccess;

struct EventPool {
  std::vector<hipEvent_t> evs;
  size_t used = 0;
  hipEvent_t get() {
    if (used == evs.size()) {
      hipEvent_t e;
      hipEventCreateWithFlags(&e, hipEventDisableTiming);
      evs.push_back(e);
    }
    return evs[used++];
  }
};
thread_local std::map<int, EventPool> tEvents;  // per device

struct Planned {
  CollOp op;
  Plan plan;
  bool memcpyOnly = false;
  bool oneRankScale = false;
  size_t copyBytes = 0;
  bool noop = false;
  bool inPlace = false;
};

// asyncMany: the group holds more than one op of this communicator; under
// MSCCL_AMD_REFERENCE_SELECTION such ops skip MSCCL as the reference's do (enqueue.cc:448-460).
ncclResult_t planOp(const CollOp& op, Planned* out, bool asyncMany) {
  ncclComm* comm = op.comm;
  out->op = op;
  int ts = refTypeSize(op.dtype);
  if (op.count == 0) { out->noop = true; return ncclSuccess; }
  if (comm->nRanks == 1) {
    if ((int)op.op >= (int)ncclNumOps) {
      // a user PreMulSum op still scales a single rank's data: the reference's oneRankReduce
      // (enqueue.cc:811-816 skips only built-in ops, onerank_reduce.cu:12-44)
      out->oneRankScale = true;
      return ncclSuccess;
    }
    // enqueue.cc:811-816: one rank = device-to-device copy (or nothing when in place)
    out->memcpyOnly = true;
    out->copyBytes = op.count * (size_t)ts;
    if (op.sendbuff == op.recvbuff) out->noop = true;
    return ncclSuccess;
  }
  CallDesc c;
  c.coll = op.coll;
  c.count = op.count;
  c.dtype = op.dtype;
  c.redop = op.devOp;
  c.nRanks = comm->nRanks;
  c.rank = comm->rank;
  c.inPlace = inPlaceOf(op.coll, op.sendbuff, op.recvbuff, op.count, op.dtype, comm->rank);
  c.customAlgo = op.customAlgo;
  c.remote = comm->anyRemote;
  out->inPlace = c.inPlace;
  return (ncclResult_t)planCall(comm->planCtx, c, asyncMany, &out->plan);
}

// Ring fallback: one workgroup per ring channel, the reference's runRing program in ring mode;
// tree fallback: two workgroups per channel (reduce up, broadcast down).
RankWork makeRingWork(Planned& p) {
  ncclComm* comm = p.op.comm;
  const int kind = p.plan.ringColl == kTreeAllReduce ? 4
                   : p.plan.ringColl == kRingAllReduce ? 0 : p.plan.ringColl == kRingReduceScatter ? 1
                   : p.inPlace ? 2 : 3;
  const DevAlgoHost& da = comm->ringAlgos[kind];
  RankWork w;
  memset(&w, 0, sizeof(w));
  w.sendbuff = p.op.sendbuff;
  w.recvbuff = p.op.recvbuff;
  w.scratch = comm->scratch;
  w.comm = comm->dComm;
  w.send = da.dSend;
  w.recv = da.dRecv;
  w.connSplit = da.connSplit;
  w.images = da.dImages;
  w.tbStride = da.tbStride;
  w.timeoutTicks = comm->timeoutTicks;
  w.llFlagMask = comm->llFlagMask;
  w.llCleanMask = comm->llCleanMask;
  w.trace = comm->dTrace;
  w.traceEvents = comm->traceEvents;
  w.npkit = comm->dNpkit;
  w.redOpArg = p.op.redArg;
  w.redOpArgIsPtr = p.op.redArgIsPtr;
  w.flags = comm->dFlags + (size_t)da.slotBase * kFlagStride;
  w.epochs = comm->dFlags + (size_t)comm->slotTotal * kFlagStride + da.slotBase;
  w.epochSlots = (int16_t)da.slotCount;
  w.maxSplit = comm->maxSplit;
  w.chunkSize = p.plan.chunkSize;
  w.minChunk = p.plan.minChunk;
  w.split = 1;
  w.merge = 1;
  w.nBlocks = (int16_t)(p.plan.ringChannels * (kind == 4 ? 2 : 1));
  w.refNthreads = (int16_t)p.plan.refNthreads;
  w.maxAllowedCount = 1;
  w.ringColl = (uint8_t)p.plan.ringColl;
  w.ringRanks = (int16_t)comm->nRanks;
  w.ringSize = p.plan.count;
  w.ringLastChunk = p.plan.ringLastChunk;
  w.launchSeq = comm->workIndex++;
  comm->last = {-1, p.plan.proto, 1, 1, p.plan.ringColl, p.plan.ringChannels, w.nBlocks};
  return w;
}

// The fold kernel (interpreter.h: runFold): the flat forms of the fallback (plan.cc:
// makeFlatTreePlan; transport.cc: ringUpload, ringAlgos[5]) or a lowered one-hop MSCCL schedule
// (lower.cc; its own fold order, foldAlgos[algoIndex]), over the flat connections.
RankWork makeFlatWork(Planned& p) {
  ncclComm* comm = p.op.comm;
  const int lowered = p.plan.algoIndex;  // -1: the fallback's flat forms
  const DevAlgoHost& da = lowered >= 0 ? comm->foldAlgos[lowered] : comm->ringAlgos[5];
  RankWork w;
  memset(&w, 0, sizeof(w));
  w.sendbuff = p.op.sendbuff;
  w.recvbuff = p.op.recvbuff;
  w.scratch = nullptr;  // the fold reads the FIFOs: no scratch
  w.comm = comm->dComm;
  w.send = da.dSend;
  w.recv = da.dRecv;
  w.connSplit = da.connSplit;  // kFlatSubs sub-connections per peer
  w.images = da.dImages;
  w.tbStride = da.tbStride;
  w.timeoutTicks = comm->timeoutTicks;
  w.llFlagMask = comm->llFlagMask;
  w.llCleanMask = comm->llCleanMask;
  w.trace = comm->dTrace;
  w.traceEvents = comm->traceEvents;
  w.npkit = comm->dNpkit;
  w.flags = comm->dFlags + (size_t)da.slotBase * kFlagStride;
  w.epochs = comm->dFlags + (size_t)comm->slotTotal * kFlagStride + da.slotBase;
  w.epochSlots = (int16_t)da.slotCount;
  w.maxSplit = comm->maxSplit;
  w.sizePerChunk = p.plan.sizePerChunk;
  w.chunkSize = p.plan.chunkSize;
  w.minChunk = p.plan.minChunk;
  w.timeoutTicks = comm->timeoutTicks;
  w.refNthreads = (int16_t)p.plan.refNthreads;
  w.foldPeers = (uint8_t)(comm->nRanks - 1);
  const int64_t pe = 16 / refTypeSize(p.plan.dtype);
  if (p.plan.lowerMode == kLowerPair) {
    // the pair kernel (interpreter.h: PairRunner) on peer record 0 of the flat connections: one
    // chunk (the whole buffer), one thread block of W workgroups, one sub-connection each; W a
    // power of two, at most flatSubs, at least kNT / 4 packs per workgroup (a function of the call
    // and the agreed flatSubs only: both ranks cut the same FIFO steps)
    const int64_t npk = (p.plan.count + pe - 1) / pe;
    int wgs = 1;
    while (wgs * 2 <= da.connSplit && npk >= (int64_t)wgs * 2 * (kNT / 4)) wgs *= 2;
    w.send = da.dSend + da.connSplit;
    w.recv = da.dRecv + da.connSplit;
    w.maxSplit = da.connSplit;  // epoch slot of workgroup k: k
    w.split = (uint8_t)wgs;
    w.nBlocks = (int16_t)wgs;
    w.merge = 1;
    w.sizePerChunk = p.plan.count;
    w.chunkSize = p.plan.count;  // one pass
    w.pairSrc = 0;
    w.pairDst = 0;
    w.pairStride = 0;
    w.pairDstBuf = (uint8_t)(p.inPlace ? 0 : 1);
    w.maxAllowedCount = 1;
    w.launchSeq = comm->workIndex++;
    comm->last = {lowered, p.plan.proto, wgs, 1, kTreeFlat, 0, w.nBlocks};
    return w;
  }
  if (p.plan.lowerMode == kLowerTwoPhase) {
    // the two-phase fold (interpreter.h: runTwoPhase): W workgroups dealing every rank's owned
    // packs M = K chunks x Q packs, at least kNT / 4 per workgroup (a function of the call and the
    // agreed flatSubs only, so every rank deals alike)
    const int64_t Q = p.plan.foldChunkPacks;
    const int64_t M = Q * (p.plan.nchunksPerLoop / comm->nRanks);
    int wgs = da.connSplit;
    while (wgs > 1 && M < (int64_t)wgs * (kNT / 4)) wgs /= 2;
    w.split = (uint8_t)wgs;
    w.nBlocks = (int16_t)wgs;
    w.merge = 1;
    w.sizePerChunk = p.plan.count;  // the whole buffer (bound of every pack)
    w.foldChunkPacks = (int32_t)Q;
    w.foldPacksPerWg = (int32_t)(M / wgs);
    w.tpOwnedPacks = (uint32_t)M;
    // m / Q as ((t + ((m - t) >> sh1)) >> sh2), t = mulhi(m, magic) (Granlund and Montgomery,
    // "Division by invariant integers using multiplication", fig. 4.1): exact for every 32-bit m
    const uint32_t d = (uint32_t)Q;
    const int l = d <= 1 ? 0 : 32 - __builtin_clz(d - 1);
    w.tpMagic = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d + 1);
    w.tpSh1 = (uint8_t)std::min(l, 1);
    w.tpSh2 = (uint8_t)std::max(l - 1, 0);
    // packs per FIFO step (kTwoPhaseStepPacks, MSCCL_AMD_TWO_PHASE_STEP): agreed knobs, so both
    // ends of every connection cut the same steps; at most a slot's
    const int64_t slotPk = comm->llSlotLines / 2;
    const int64_t stepPk = comm->knobs.twoPhaseStep > 0 ? comm->knobs.twoPhaseStep : kTwoPhaseStepPacks;
    w.tpStepPacks = (uint16_t)std::max<int64_t>(64, std::min<int64_t>({stepPk, slotPk, 65535}));
    w.ringColl = 0;
    w.foldChunkPacks = (int32_t)Q;
    w.maxAllowedCount = 1;
    w.launchSeq = comm->workIndex++;
    comm->last = {lowered, p.plan.proto, wgs, 1, kTreeFlat, 0, w.nBlocks};
    return w;
  }
  // workgroups per rank: one per kFoldPacksPerWg packs of the call, at most kFlatSubs (a function
  // of the call's size alone, so every rank picks the same and the two ends of every
  // sub-connection own the same packs; one workgroup against up to four: profiles/r03_ab_fold_wgs_and_r02.txt; 16 against 4: r04t_lat.txt)
  const int64_t npk = (p.plan.sizePerChunk + pe - 1) / pe;
  const int wgs = (int)std::max<int64_t>(1, std::min<int64_t>(kFlatSubs, (npk + kFoldPacksPerWg - 1) / kFoldPacksPerWg));
  w.split = (uint8_t)wgs;
  w.foldPacksPerWg = (int32_t)(npk / wgs);
  w.maxOpElems = (int64_t)kMaxRunSlots * (comm->llSlotLines / 2) * pe;
  int merge = 1;
  if (p.plan.nIters > 1 && p.plan.maxAllowedCount == 1) {  // makeWork's rule, send runs of one chunk
    const int64_t chunk = std::max<int64_t>(1, p.plan.chunkSize);
    merge = (int)std::max<int64_t>(1, std::min<int64_t>(64, w.maxOpElems / chunk));
  }
  w.merge = (uint8_t)merge;
  w.nBlocks = (int16_t)wgs;  // mscclFoldKernel (interpreter.h: runFold)
  // the kernel's collective: 0 the flat tree's AllReduce, else kRingReduceScatter / kRingAllGather
  w.ringColl = (uint8_t)(p.plan.flatColl == kRingAllReduce ? 0 : p.plan.flatColl);
  w.foldPeers = (uint8_t)(comm->nRanks - 1);
  w.foldChunkPacks = (int32_t)p.plan.foldChunkPacks;
  w.refNthreads = (int16_t)p.plan.refNthreads;
  w.maxAllowedCount = (uint8_t)p.plan.maxAllowedCount;
  w.launchSeq = comm->workIndex++;
  comm->last = {lowered, p.plan.proto, wgs, merge, kTreeFlat, 0, w.nBlocks};
  return w;
}

// The direct form of a Simple schedule (interpreter.h: DirectRunner; lower.h: DirectLowering):
// launchGroup runs it when every rank of the communicator is in the launch.  No connection, flag
// or epoch is touched (a later interpreted call of the schedule finds them as the last one left
// them).  Workgroups per rank: MSCCL_AMD_DIRECT_WGS per GPU over the ranks, at most 255
// (RankWork::split is a byte), and no more than keep 4 packs per lane (the kernel's
// MSCCL_DIRECT_UD).  No workgroup waits on another, so they need not all be resident.  Default
// 1024 for the AllGather / AllReduce, 512 for the ReduceScatter, whose lanes already hold n
// loads per pack (8 co-resident ranks, same box, 512 / 1024 / 2048: AG 0.109 / 0.102 / 0.150 ms,
// RS 0.125 / 0.135 / 0.141, C4 0.809 / 0.802 / 0.935; profiles/r06g_c45_w*.json).
RankWork makeDirectWork(Planned& p) {
  ncclComm* comm = p.op.comm;
  const int g = p.plan.algoIndex;  // -1: the ring fallback's ReduceScatter / AllGather (plan.cc: planCall)
  const DevAlgoHost& da = g >= 0 ? comm->directAlgos[g] : comm->ringDirectRS;
  const int coll = g >= 0 ? comm->algoDirect[g].coll : p.plan.ringColl == kRingAllGather ? kAllGather : kReduceScatter;
  const int n = comm->nRanks;
  RankWork w;
  memset(&w, 0, sizeof(w));
  w.sendbuff = p.op.sendbuff;
  w.recvbuff = p.op.recvbuff;
  w.comm = comm->dComm;
  w.images = da.dImages;
  w.tbStride = da.tbStride;
  w.timeoutTicks = comm->timeoutTicks;
  w.llFlagMask = comm->llFlagMask;
  w.llCleanMask = comm->llCleanMask;
  w.refNthreads = (int16_t)p.plan.refNthreads;
  w.ringColl = (uint8_t)(coll == kAllGather ? kRingAllGather : coll == kReduceScatter ? kRingReduceScatter : kRingAllReduce);
  w.sizePerChunk = p.plan.count;  // one rank block: AG input bytes, RS output elements, AR elements
  const int64_t pe = 16 / refTypeSize(p.plan.dtype);
  const int64_t packs = (p.plan.count + pe - 1) / pe;
  const int64_t share = coll == kAllReduce ? (packs + n - 1) / n : packs;
  static const int64_t envTarget = envInt("MSCCL_AMD_DIRECT_WGS", 0);
  const int64_t target = envTarget > 0 ? envTarget : coll == kReduceScatter ? 512 : 1024;
  const int64_t perWg = (int64_t)kNT * 4;
  const int wgs = (int)std::max<int64_t>(1, std::min<int64_t>({target / n, (int64_t)255, (share + perWg - 1) / perWg}));
  w.split = (uint8_t)wgs;
  w.nBlocks = (int16_t)wgs;
  w.merge = 1;
  w.maxAllowedCount = 1;
  const uint32_t d = (uint32_t)p.plan.directChunkPacks;  // packs per output chunk (0: one class)
  w.foldChunkPacks = (int32_t)d;
  if (d > 0) {
    const int l = d <= 1 ? 0 : 32 - __builtin_clz(d - 1);  // the two-phase fold's division (makeFlatWork)
    w.tpMagic = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d + 1);
    w.tpSh1 = (uint8_t)std::min(l, 1);
    w.tpSh2 = (uint8_t)std::max(l - 1, 0);
  }
  w.directRank = (int16_t)comm->rank;
  w.launchSeq = comm->workIndex++;
  comm->last = {g, p.plan.proto, wgs, 1, 0, 0, w.nBlocks};
  return w;
}

RankWork makeWork(Planned& p) {
  if (p.plan.ringColl == kTreeFlat) return makeFlatWork(p);
  if (p.plan.ringColl) return makeRingWork(p);
  ncclComm* comm = p.op.comm;
  const DevAlgoHost& da = comm->devAlgos[p.plan.algoIndex];
  RankWork w;
  memset(&w, 0, sizeof(w));
  w.sendbuff = p.op.sendbuff;
  w.recvbuff = p.op.recvbuff;
  w.scratch = comm->scratch;
  w.comm = comm->dComm;
  w.send = da.dSend;
  w.recv = da.dRecv;
  w.connSplit = da.connSplit;
  w.images = da.dImages;
  w.tbStride = da.tbStride;
  w.timeoutTicks = comm->timeoutTicks;
  w.llFlagMask = comm->llFlagMask;
  w.llCleanMask = comm->llCleanMask;
  w.trace = comm->dTrace;
  w.traceEvents = comm->traceEvents;
  w.npkit = comm->dNpkit;
  w.redOpArg = p.op.redArg;
  w.redOpArgIsPtr = p.op.redArgIsPtr;
  w.flags = comm->dFlags + (size_t)da.slotBase * kFlagStride;
  w.epochs = comm->dFlags + (size_t)comm->slotTotal * kFlagStride + da.slotBase;
  w.epochSlots = (int16_t)da.slotCount;
  w.maxSplit = comm->maxSplit;
  w.sizePerChunk = p.plan.sizePerChunk;
  w.chunkSize = p.plan.chunkSize;
  w.minChunk = p.plan.minChunk;
  // Workgroups of a split thread block own 16-B pack positions inside each chunk, so a split
  // needs whole packs per chunk; sizePerChunk is identical on every rank, so all ranks agree.
  int split = comm->algoSplit.empty() ? 1 : comm->algoSplit[p.plan.algoIndex];
  const int64_t pe = 16 / refTypeSize(p.plan.dtype);
  if (p.plan.sizePerChunk % pe != 0) split = 1;
  // Small messages: fewer, fuller workgroups, at least one pack per 4 lanes of every workgroup
  // (C2 pair schedule: 128 KiB 9.4 -> 8.4 us, 512 KiB 9.6 -> 8.9 us against one pack per lane;
  // below that more workgroups only add launch and poll overhead); a split forced with
  // MSCCL_AMD_SPLIT is kept as is.
  if (comm->knobs.split <= 0)
    while (split > 1 && p.plan.sizePerChunk / pe < (int64_t)split * (kNT / 4)) split /= 2;
  // the wide budget (two co-resident LL ranks, plan.h: kWideSplitMinBytes) only while every
  // workgroup still moves kWideSplitMinBytes of the call.  Both inputs must be the same on every
  // rank: nBytes is, and the thread-block count is the most over every rank's program
  // (algoMaxBlocks, agreed at init) -- ranks of one schedule may run different numbers of thread
  // blocks (topo.cc:1174-1184), and this rank's own count would let the two ends of a
  // sub-connection step back differently
  if ((size_t)p.plan.algoIndex < comm->algoSplitBase.size())
    while (split > comm->algoSplitBase[p.plan.algoIndex] &&
           p.plan.nBytes < (int64_t)comm->algoMaxBlocks[p.plan.algoIndex] * split * kWideSplitMinBytes)
      split /= 2;
  w.split = (uint8_t)split;
  w.nBlocks = (int16_t)(da.nBlocks * split);
  // Consecutive full interpreter iterations can run as one: every element still sees the same
  // operations in the same order (only a partial last iteration can take the per-element reduce
  // path, and it stays an iteration of its own).  Primitive calls are cut into FIFO-slot steps on
  // the device, so any merge fits; by default every full iteration runs in one op (fewest
  // dependency rounds).  maxAllowedCount is 1 whenever there is more than one iteration, so one
  // op never exceeds one chunk.
  // Merged calls keep every run of sends before a receive within kMaxRunSlots FIFO slots per
  // sub-connection (devcomm.h); a workgroup moves 1/split of a call.  sendRun = the schedule's
  // longest such run in chunks (algoSendRun).
  int64_t slotPacks;
  if (p.plan.proto == kProtoSimple) slotPacks = comm->simpleSlotBytes / 16;
  else if (p.plan.proto == kProtoLL128) slotPacks = (int64_t)(comm->llSlotLines / 256) * 64 * 3;
  else slotPacks = comm->llSlotLines / 2;
  w.maxOpElems = (int64_t)kMaxRunSlots * slotPacks * pe * split;
  const int64_t sendRun = std::max(1, comm->algoSendRun.empty() ? 1 : comm->algoSendRun[p.plan.algoIndex]);
  int merge = 1;
  if (p.plan.nIters > 1 && p.plan.maxAllowedCount == 1) {
    const int64_t envMerge = comm->knobs.merge;
    // as many full iterations per call as the bound allows: fewest dependency rounds
    // (C2 32 MiB LL: 348 GB/s with `split` iterations per call, 405 with all 16)
    const int64_t chunk = std::max<int64_t>(1, p.plan.chunkSize);
    // A schedule in pair form on every rank (transport.cc: pairFormOf; init.cc: algoPairAll):
    // every thread block sends one chunk to its peer and receives one from it.  Its run of sends
    // may fill the whole FIFO (kLLFifoSlots, not kMaxRunSlots): both ends' runs fit at once even
    // when a rank runs the general kernel, which does not fuse and sends the run before receiving
    // (a run past the FIFO deadlocks against the peer's, profiles/r05am_pair_merge.txt), and a
    // rank's next launch only waits for the peer to drain this one.  C2 32 MiB: 64 iterations of
    // 8 slots per workgroup, one pass on the pair kernel instead of two.
    const bool pairForm = p.plan.proto == kProtoLL && (size_t)p.plan.algoIndex < comm->algoPairAll.size() &&
                          comm->algoPairAll[p.plan.algoIndex];
    const int64_t runElems = pairForm ? w.maxOpElems / kMaxRunSlots * kLLFifoSlots : w.maxOpElems;
    const int64_t fit = std::max<int64_t>(1, runElems / (chunk * sendRun));
    merge = (int)std::min<int64_t>(envMerge > 0 ? envMerge : fit, fit);  // MSCCL_AMD_MERGE only lowers it
    // a merged iteration stays within 1 GiB, far inside a buffer descriptor's 2 GiB reach
    const int64_t reach = std::max<int64_t>(1, (1ll << 30) / (chunk * refTypeSize(p.plan.dtype)));
    merge = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)merge, 64, reach}));
  }
  w.merge = (uint8_t)merge;
  w.refNthreads = (int16_t)p.plan.refNthreads;
  w.maxAllowedCount = (uint8_t)p.plan.maxAllowedCount;
  w.pairSrc = -1;
  if ((size_t)p.plan.algoIndex < comm->algoPair.size() && p.plan.proto == kProtoLL) {
    const ncclComm::PairForm& pf = comm->algoPair[p.plan.algoIndex];
    w.pairSrc = (int16_t)pf.src;
    w.pairDst = (int16_t)pf.dst;
    w.pairStride = (int16_t)pf.stride;
    w.pairDstBuf = (uint8_t)pf.dstBuf;
  }
  w.launchSeq = comm->workIndex++;
  comm->last = {p.plan.algoIndex, p.plan.proto, split, merge, 0, 0, w.nBlocks};
  return w;
}

// mscclSmallKernel takes a call whose LL interpreter loop runs in equal passes (one iteration,
// or full iterations merged with none left over) of an MSCCL schedule, without trace or NPKit
// log, with a Sum..Min op (interpreter.h: runSmall).  Both kernels cut a
// transfer into the same primitive calls, so ranks that choose differently still agree.
// chunks any transfer offset of the algorithm can reach (the loader bounds offsets by the
// buffers' chunk counts, topo.cc:725)
int64_t maxChunkIndex(const Algorithm& a, int64_t ncpl) {
  return std::max<int64_t>({ncpl, (int64_t)a.nInputChunks, (int64_t)a.nOutputChunks, (int64_t)a.nScratchChunks});
}

bool smallEligible(const Planned& p, const RankWork& w) {
  const ncclComm* comm = p.op.comm;
  // run()'s loop in equal passes: a single iteration, or full iterations merged `merge` at a
  // time with none left over (interpreter.h: run, runSmall)
  const int64_t sp = p.plan.sizePerChunk, cs = p.plan.chunkSize;
  const int64_t k = cs > 0 ? sp / cs : 0, m = std::min<int64_t>(std::max<int>(1, w.merge), std::max<int64_t>(1, k));
  const bool onePass = sp <= cs || (cs > 0 && sp % cs == 0 && k % m == 0);
  const bool flat = p.plan.ringColl == kTreeFlat;
  // the ring fallback's one-iteration calls (interpreter.h: runSmall's ring pass): runRing's loop
  // covers the call once (AllReduce: nChannels * nRanks * chunkSize, ReduceScatter / AllGather:
  // nChannels * chunkSize elements), every offset within 32 bits
  const bool ring = p.plan.ringColl == kRingAllReduce || p.plan.ringColl == kRingReduceScatter ||
                    p.plan.ringColl == kRingAllGather;
  if (ring) {
    const int64_t loop = (int64_t)w.nBlocks * cs * (p.plan.ringColl == kRingAllReduce ? w.ringRanks : 1);
    const int64_t span = (int64_t)w.ringRanks * w.ringSize * refTypeSize(p.plan.dtype);
    if (cs <= 0 || w.ringSize > loop || span > (1ll << 30) || w.split != 1) return false;
  }
  if (!comm->knobs.smallKernel || !(p.plan.ringColl == 0 || flat || ring) || p.plan.proto != kProtoLL ||
      p.op.devOp > 3 || !onePass || !(w.trace == nullptr || comm->traceLight) || w.npkit != nullptr ||
      (w.split & (w.split - 1)) != 0)
    return false;
  if (ring) return true;
  // (ring / tree plans have no algorithm: algoIndex -1 is only read past the checks above)
  const int64_t chunks = flat ? 1 : maxChunkIndex(comm->algos[p.plan.algoIndex], p.plan.nchunksPerLoop);
  return p.plan.sizePerChunk * chunks * refTypeSize(p.plan.dtype) <= (1ll << 30);  // runSmall's 32-bit offsets
}

// The direct form runs when every op of the launch may (Plan::directOk: the same schedule) and the
// launch holds every rank of one clique (ncclComm::clique) once: then all of them are in this
// launch, whose start follows every rank's stream, and the argument block, in rank order, gives
// every rank's buffers.  The decision is the same for every rank (they are all here).
bool directLaunch(std::vector<Planned*>& ps) {
  const ncclComm* c0 = ps[0]->op.comm;
  if (c0->clique == 0 || (int)ps.size() != c0->nRanks) return false;
  std::vector<bool> seen(c0->nRanks, false);
  for (const Planned* p : ps) {
    const ncclComm* c = p->op.comm;
    if (!p->plan.directOk || c->clique != c0->clique || p->plan.algoIndex != ps[0]->plan.algoIndex ||
        p->op.coll != ps[0]->op.coll || p->op.count != ps[0]->op.count || seen[c->rank])
      return false;
    seen[c->rank] = true;
  }
  std::sort(ps.begin(), ps.end(), [](const Planned* a, const Planned* b) { return a->op.comm->rank < b->op.comm->rank; });
  return true;
}

ncclResult_t launchGroup(std::vector<Planned*>& ps) {
  const bool direct = directLaunch(ps);  // (sorts ps by rank when true)
  ncclComm* c0 = ps[0]->op.comm;
  int dev = c0->cudaDev;
  hipStream_t primary = ps[0]->op.stream;
  LaunchArgs args;
  memset(&args, 0, sizeof(args));
  int blocks = 0;
  bool small = !direct;
  for (size_t i = 0; i < ps.size(); i++) {
    RankWork w = direct ? makeDirectWork(*ps[i]) : makeWork(*ps[i]);
    w.blockBase = (int16_t)blocks;
    blocks += w.nBlocks;
    args.w[i] = w;
    small = small && smallEligible(*ps[i], w);
  }
  args.nRanks = (int)ps.size();
  if (blocks == 0) return ncclSuccess;
  EventPool& pool = tEvents[dev];
  pool.used = 0;
  for (size_t i = 1; i < ps.size(); i++) {
    if (ps[i]->op.stream != primary) {
      hipEvent_t e = pool.get();
      hipEventRecord(e, ps[i]->op.stream);
      hipStreamWaitEvent(primary, e, 0);
    }
  }
  const Planned& p0 = *ps[0];
  // a launch group holds flat works of one lowering mode only, or none (executeOps keys launches
  // on it): the fold, the pair kernel on the flat connections, or the two-phase fold
  const bool flatWork = !direct && p0.plan.ringColl == kTreeFlat;
  const bool fold = flatWork && p0.plan.lowerMode == kLowerFold;
  const bool lowPair = flatWork && p0.plan.lowerMode == kLowerPair;
  const bool two = flatWork && p0.plan.lowerMode == kLowerTwoPhase;
  // the small kernel holding only the exchange's transfers when every work of the launch needs
  // no more (devcomm.h: kSetExchange)
  int set = kSetExchange;
  for (Planned* p : ps) {
    const ncclComm* c = p->op.comm;
    if (p->plan.ringColl != 0 || (size_t)p->plan.algoIndex >= c->algoSet.size() || c->algoSet[p->plan.algoIndex] != kSetExchange)
      set = kSetAll;
  }
  // the pair kernel (interpreter.h: PairRunner) when every work is a pair-form schedule whose call
  // is one pass of runSmall's loop, untraced
  bool pair = small && !flatWork && set == kSetExchange && p0.op.comm->knobs.pairKernel;
  for (int i = 0; i < args.nRanks && pair; i++) {
    const RankWork& w = args.w[i];
    pair = w.pairSrc >= 0 && w.trace == nullptr && w.sizePerChunk <= w.chunkSize * std::max<int>(1, w.merge);
  }
  // (the lowered pair runs the pair kernel whatever MSCCL_AMD_PAIR_KERNEL says: both ends of its
  // flat connections run it, the plan being the same on every rank)
  pair = !direct && (pair || lowPair);
  LaunchFn fn = direct ? getDirectLaunchFn(p0.plan.dtype, p0.op.devOp)
                : fold ? getFoldLaunchFn(p0.plan.dtype, p0.op.devOp)
                : two ? getTwoPhaseLaunchFn(p0.plan.dtype, p0.op.devOp)
                : pair ? getPairLaunchFn(p0.plan.dtype, p0.op.devOp)
                : small ? getSmallLaunchFn(p0.plan.dtype, p0.op.devOp, set)
                        : getLaunchFn(p0.plan.dtype, p0.op.devOp, p0.plan.proto);
  for (Planned* p : ps) {
    // small: 0 the general kernel, 1 the small-call kernel, 2 a flat kernel (fold, lowered pair,
    // two-phase); kernel: 0 general, 1 small, 2 fold, 3 pair, 4 two-phase
    p->op.comm->last.small = flatWork ? 2 : small ? 1 : 0;
    p->op.comm->last.set = small && !flatWork ? set : 0;
    p->op.comm->last.pair = pair ? 1 : 0;
    p->op.comm->last.kernel = direct ? 5 : fold ? 2 : two ? 4 : pair ? 3 : small ? 1 : 0;
  }
  if (!fn) { WARN("MSCCL: no kernel for type %d op %d proto %d", p0.plan.dtype, p0.op.devOp, p0.plan.proto); return ncclInvalidArgument; }
  if (!direct) {
    // Every workgroup of the launch may spin on every other one (FIFO credits, dependency
    // flags), so all of them must be resident at once: refuse what the GPU cannot hold instead
    // of launching a grid that can only hang.  (The direct kernel's workgroups wait on nothing.)
    static std::map<std::pair<int, LaunchFn>, int> cap;
    auto key = std::make_pair(dev, fn);
    auto it = cap.find(key);
    if (it == cap.end()) {
      int cus = 0;
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      it = cap.emplace(key, cus * fn(args, kQueryResidency, nullptr)).first;
    }
    if (it->second > 0 && blocks > it->second) {
      WARN("MSCCL: launch needs %d co-resident workgroups but device %d holds %d of this kernel at once "
           "(fewer co-resident ranks, fewer thread blocks or MSCCL_AMD_SPLIT=1)", blocks, dev, it->second);
      return ncclInvalidUsage;
    }
  }
  if (fn(args, blocks, (void*)primary) != 0) {
    WARN("MSCCL: kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
    return ncclUnhandledCudaError;
  }
  for (size_t i = 1; i < ps.size(); i++) {
    if (ps[i]->op.stream != primary) {
      hipEvent_t e = pool.get();
      hipEventRecord(e, primary);
      hipStreamWaitEvent(ps[i]->op.stream, e, 0);
    }
  }
  return ncclSuccess;
}

}  // namespace

bool groupActive() { return tGroupDepth > 0; }
void groupAddInit(std::function<ncclResult_t()> fn, ncclComm* comm) { tInits.emplace_back(std::move(fn), comm); }
void groupAddOp(const CollOp& op) { tOps.push_back(op); }

ncclResult_t executeOps(std::vector<CollOp>& ops) {
  // rounds: the k-th op of every communicator runs in round k.  The usual group holds one op per
  // communicator (one round); nothing here allocates per call beyond the per-round vectors.
  std::vector<ncclComm*> order;
  std::vector<std::vector<size_t>> perComm;  // parallel to `order`
  order.reserve(ops.size());
  for (size_t i = 0; i < ops.size(); i++) {
    size_t j = 0;
    while (j < order.size() && order[j] != ops[i].comm) j++;
    if (j == order.size()) {
      order.push_back(ops[i].comm);
      perComm.emplace_back();
    }
    perComm[j].push_back(i);
  }
  size_t rounds = 0;
  for (auto& v : perComm) rounds = std::max(rounds, v.size());
  int saved = 0;
  hipGetDevice(&saved);
  int cur = saved;
  auto setDev = [&cur](int d) {
    if (d != cur) {
      hipSetDevice(d);
      cur = d;
    }
  };
  ncclResult_t res = ncclSuccess;
  for (size_t k = 0; k < rounds && res == ncclSuccess; k++) {
    std::vector<Planned> planned;
    planned.reserve(order.size());
    for (size_t j = 0; j < order.size(); j++) {
      auto& v = perComm[j];
      if (k >= v.size()) continue;
      planned.emplace_back();
      res = planOp(ops[v[k]], &planned.back(), v.size() > 1);
      if (res != ncclSuccess) break;
    }
    if (res != ncclSuccess) break;
    // copies / one-rank scaling run at once; kernels are fused per (device, type, op, protocol)
    typedef std::tuple<int, int, int, int, int> LaunchKey;  // + flat kind: 0 none, 1 + lowerMode (own kernels)
    std::vector<std::pair<LaunchKey, std::vector<Planned*>>> launches;
    for (auto& p : planned) {
      if (p.noop) continue;
      setDev(p.op.comm->cudaDev);
      if (p.memcpyOnly) {
        if (hipMemcpyAsync(p.op.recvbuff, p.op.sendbuff, p.copyBytes, hipMemcpyDeviceToDevice, p.op.stream) != hipSuccess) {
          res = ncclUnhandledCudaError;
          break;
        }
        continue;
      }
      if (p.oneRankScale) {
        OneRankFn f = getOneRankFn((int)p.op.dtype);
        if (!f || f(p.op.sendbuff, p.op.recvbuff, p.op.count, p.op.redArg, p.op.redArgIsPtr, (void*)p.op.stream) != 0) {
          res = ncclUnhandledCudaError;
          break;
        }
        continue;
      }
      const LaunchKey key =
          std::make_tuple(p.op.comm->cudaDev, p.plan.dtype, p.op.devOp, p.plan.proto,
                          p.plan.ringColl == kTreeFlat ? 1 + p.plan.lowerMode : 0);
      size_t j = 0;
      while (j < launches.size() && launches[j].first != key) j++;
      if (j == launches.size()) launches.emplace_back(key, std::vector<Planned*>());
      launches[j].second.push_back(&p);
    }
    for (auto& kv : launches) {
      if (res != ncclSuccess) break;
      auto& list = kv.second;
      setDev(std::get<0>(kv.first));
      if (list.size() > (size_t)kMaxLaunchRanks) {
        // the ranks' workgroups wait on each other: launched in parts they could only time out
        WARN("MSCCL: %zu co-resident ranks on device %d in one group; one launch carries at most %d",
             list.size(), std::get<0>(kv.first), kMaxLaunchRanks);
        res = ncclInvalidUsage;
        break;
      }
      res = launchGroup(list);
    }
  }
  setDev(saved);
  return res;
}

}  // namespace msccl

using namespace msccl;

namespace {

// IEEE binary16 of a float, round to nearest even (__float2half); the host compiler has no
// _Float16.  Normal and subnormal results, overflow to infinity, NaN kept quiet.
uint16_t floatToHalfRne(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const uint32_t ax = x & 0x7fffffffu;
  if (ax >= 0x7f800000u) return (uint16_t)(sign | 0x7c00u | (ax > 0x7f800000u ? 0x200u : 0));
  if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  // rounds to >= 65520: infinity
  if (ax < 0x38800000u) {                                      // subnormal or zero half
    if (ax < 0x33000000u) return (uint16_t)sign;               // at most half the smallest subnormal
    const uint32_t m = (ax & 0x7fffffu) | 0x800000u;           // value = m * 2^(e - 150)
    const int s = 126 - (int)(ax >> 23);                       // half subnormal = value * 2^24 = m >> s
    uint32_t h = m >> s;
    const uint32_t rem = m & ((1u << s) - 1), halfway = 1u << (s - 1);
    if (rem > halfway || (rem == halfway && (h & 1u))) h++;    // may carry into the smallest normal
    return (uint16_t)(sign | h);
  }
  const uint32_t e = (ax >> 23) - 112, m = ax & 0x7fffffu;
  uint32_t h = (e << 10) | (m >> 13);
  const uint32_t rem = m & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
  return (uint16_t)(sign | h);
}

// ncclUserRedOpMangle (comm.h:223-235): user op ids are ncclNumOps + index, xor-ed with a hash
// of the communicator so an op from another communicator is rejected; an involution.
ncclRedOp_t userRedOpMangle(const ncclComm* comm, ncclRedOp_t op) {
  if ((int)op < (int)ncclNumOps) return op;
  uint64_t h = reinterpret_cast<uint64_t>(comm);
  h ^= h >> 32;
  h *= 0x9e3779b97f4a7c13ull;
  h >>= 32;
  h &= (uint64_t)ncclMaxRedOp;
  const int op1 = (int)h ^ (int)op;
  return op1 < (int)ncclNumOps ? op : (ncclRedOp_t)op1;
}

// hostToDevRedOp (enqueue.cc:1388-1454): the device operation of a call.  ncclAvg is a sum of
// inputs pre-multiplied by 1/nRanks (rounded to the element type) for floating types, and a
// sum divided by nRanks afterwards for integer types.
ncclResult_t hostToDevRedOp(ncclComm* comm, ncclRedOp_t op, ncclDataType_t dt, CollOp* o, const char* name) {
  o->redArg = 0;
  o->redArgIsPtr = 0;
  if ((int)op < (int)ncclAvg) {
    o->devOp = (int)op;
    return ncclSuccess;
  }
  if (op == ncclAvg) {
    const int n = comm->nRanks;
    switch (dt) {
      case ncclInt8: case ncclUint8: case ncclInt32: case ncclUint32: case ncclInt64: case ncclUint64:
        o->devOp = kDevSumPostDiv;
        o->redArg = (uint64_t)n;
        break;
      case ncclFloat16: {
        const uint16_t s = floatToHalfRne((float)(1.0 / n));  // __float2half(float(1.0/n))
        memcpy(&o->redArg, &s, 2);
        o->devOp = kDevPreMulSum;
        break;
      }
      case ncclBfloat16: {
        const float f = (float)(1.0 / n);              // __float2bfloat16(float(1.0/n)): RNE
        uint32_t u;
        memcpy(&u, &f, 4);
        const uint16_t b = (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
        memcpy(&o->redArg, &b, 2);
        o->devOp = kDevPreMulSum;
        break;
      }
      case ncclFloat32: {
        const float f = (float)(1.0 / n);
        memcpy(&o->redArg, &f, 4);
        o->devOp = kDevPreMulSum;
        break;
      }
      default: {  // ncclFloat64
        const double d = 1.0 / n;
        memcpy(&o->redArg, &d, 8);
        o->devOp = kDevPreMulSum;
        break;
      }
    }
    return ncclSuccess;
  }
  const int ix = (int)userRedOpMangle(comm, op) - (int)ncclNumOps;
  if (ix < 0 || ix >= (int)comm->userRedOps.size() || comm->userRedOps[ix].freeNext != -1) {
    WARN("%s : reduction operation %d unknown to this communicator", name, (int)op);
    return ncclInvalidArgument;
  }
  const ncclComm::UserRedOp& u = comm->userRedOps[ix];
  if (u.datatype != dt) {
    WARN("Data type supplied to user-created ncclRedOp_t does not match type given to reduction operation");
    return ncclInvalidArgument;
  }
  o->devOp = kDevPreMulSum;
  o->redArg = u.scalarArg;
  o->redArgIsPtr = u.argIsPtr ? 1 : 0;
  return ncclSuccess;
}

ncclResult_t enqueue(ncclComm* comm, int coll, const void* sendbuff, void* recvbuff, size_t count,
                     ncclDataType_t dtype, ncclRedOp_t op, hipStream_t stream, int customAlgo, const char* name) {
  if (!commValid(comm)) { WARN("%s : invalid communicator", name); return ncclInvalidArgument; }
  if (comm->hostErr != nullptr && __atomic_load_n(comm->hostErr, __ATOMIC_ACQUIRE) != kDevOk) {
    // A kernel of this communicator timed out or was aborted and drained: its FIFO step
    // counters no longer match the peers', so nothing more may run on it.
    WARN("%s : communicator has an asynchronous error (%u); destroy or abort it", name,
         __atomic_load_n(comm->hostErr, __ATOMIC_ACQUIRE));
    return ncclSystemError;
  }
  if ((int)dtype < 0 || (int)dtype >= ncclNumTypes) { WARN("%s : invalid type %d", name, (int)dtype); return ncclInvalidArgument; }
  if ((int)op < 0 || (int)op > (int)ncclMaxRedOp) { WARN("%s : invalid reduction operation %d", name, (int)op); return ncclInvalidArgument; }
  if (count > 0 && (sendbuff == nullptr || recvbuff == nullptr)) { WARN("%s : buffer argument is NULL", name); return ncclInvalidArgument; }
  CollOp o{comm, coll, sendbuff, recvbuff, count, dtype, op, stream, customAlgo};
  NCCLCHECK(hostToDevRedOp(comm, op, dtype, &o, name));
  if (groupActive()) {
    groupAddOp(o);
    return ncclSuccess;
  }
  std::vector<CollOp> v{o};
  return executeOps(v);
}

}  // namespace

extern "C" {

ncclResult_t ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                           ncclRedOp_t op, ncclComm_t comm, hipStream_t stream) {
  return enqueue(comm, kAllReduce, sendbuff, recvbuff, count, datatype, op, stream, -1, "AllReduce");
}

ncclResult_t ncclReduceScatter(const void* sendbuff, void* recvbuff, size_t recvcount, ncclDataType_t datatype,
                               ncclRedOp_t op, ncclComm_t comm, hipStream_t stream) {
  return enqueue(comm, kReduceScatter, sendbuff, recvbuff, recvcount, datatype, op, stream, -1, "ReduceScatter");
}

ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount, ncclDataType_t datatype,
                           ncclComm_t comm, hipStream_t stream) {
  return enqueue(comm, kAllGather, sendbuff, recvbuff, sendcount, datatype, ncclSum, stream, -1, "AllGather");
}

ncclResult_t ncclAllToAll(const void* sendbuff, void* recvbuff, size_t sendcount, ncclDataType_t datatype,
                          ncclComm_t comm, hipStream_t stream) {
  return enqueue(comm, kAllToAll, sendbuff, recvbuff, sendcount, datatype, ncclSum, stream, -1, "AllToAll");
}

ncclResult_t ncclCustomCollective(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                                  int mscclAlgorithmIndex, ncclComm_t comm, hipStream_t stream) {
  return enqueue(comm, kCustom, sendbuff, recvbuff, count, datatype, ncclSum, stream, mscclAlgorithmIndex,
                 "CustomCollective");
}

ncclResult_t ncclRedOpCreatePreMulSum(ncclRedOp_t* op, void* scalar, ncclDataType_t datatype,
                                      ncclScalarResidence_t residence, ncclComm_t comm) {
  if (!commValid(comm) || op == nullptr || scalar == nullptr) return ncclInvalidArgument;
  if ((int)datatype < 0 || (int)datatype >= ncclNumTypes) return ncclInvalidArgument;
  if (comm->userRedOpFreeHead == (int)comm->userRedOps.size()) {  // grow the free list
    const int cap = std::max<int>(4, 2 * (int)comm->userRedOps.size());
    const int old = (int)comm->userRedOps.size();
    comm->userRedOps.resize(cap);
    for (int i = old; i < cap; i++) comm->userRedOps[i].freeNext = i + 1;
  }
  const int ix = comm->userRedOpFreeHead;
  ncclComm::UserRedOp& u = comm->userRedOps[ix];
  comm->userRedOpFreeHead = u.freeNext;
  u.freeNext = -1;
  u.datatype = datatype;
  u.scalarArg = 0;
  if (residence == ncclScalarHostImmediate) {
    u.argIsPtr = false;
    memcpy(&u.scalarArg, scalar, (size_t)refTypeSize((int)datatype));
  } else {
    u.argIsPtr = true;
    u.scalarArg = reinterpret_cast<uint64_t>(scalar);
  }
  *op = userRedOpMangle(comm, (ncclRedOp_t)((int)ncclNumOps + ix));
  return ncclSuccess;
}

ncclResult_t ncclRedOpDestroy(ncclRedOp_t op, ncclComm_t comm) {
  if (0 <= (int)op && (int)op < (int)ncclNumOps) {
    WARN("ncclRedOpDestroy : operator is a NCCL builtin.");
    return ncclInvalidArgument;
  }
  if ((int)op < 0 || (int)ncclMaxRedOp < (int)op) {
    WARN("ncclRedOpDestroy :  operator is garbage.");
    return ncclInvalidArgument;
  }
  if (!commValid(comm)) return ncclInvalidArgument;
  const int ix = (int)userRedOpMangle(comm, op) - (int)ncclNumOps;
  if (ix < 0 || ix >= (int)comm->userRedOps.size() || comm->userRedOps[ix].freeNext != -1) {
    WARN("ncclRedOpDestroy : operator unknown to this communicator.");
    return ncclInvalidArgument;
  }
  comm->userRedOps[ix].freeNext = comm->userRedOpFreeHead;
  comm->userRedOpFreeHead = ix;
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
  if (tGroupDepth == 0) tGroupError = ncclSuccess;
  tGroupDepth++;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  if (tGroupDepth == 0) { WARN("ncclGroupEnd: not in a group call."); return ncclInvalidUsage; }
  if (--tGroupDepth > 0) return ncclSuccess;
  ncclResult_t res = ncclSuccess;
  if (!tInits.empty()) {
    auto inits = std::move(tInits);
    tInits.clear();
    std::vector<ncclResult_t> rs(inits.size(), ncclSuccess);
    std::vector<std::thread> th;
    int dev = 0;
    hipGetDevice(&dev);
    for (size_t i = 0; i < inits.size(); i++)
      th.emplace_back([&, i]() {
        hipSetDevice(inits[i].second->cudaDev);
        rs[i] = inits[i].first();
      });
    for (auto& t : th) t.join();
    hipSetDevice(dev);
    for (auto r : rs)
      if (r != ncclSuccess) res = r;
  }
  if (!tOps.empty()) {
    auto ops = std::move(tOps);
    tOps.clear();
    ncclResult_t r = executeOps(ops);
    if (r != ncclSuccess) res = r;
  }
  return res;
}

}  // extern "C"

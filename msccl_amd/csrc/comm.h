// Host communicator (replaces the reference's struct ncclComm, include/comm.h:95-217, for the
// single-node MSCCL path only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <memory>
#include <string>
#include <vector>

#include "../../include/nccl.h"
#include "algo.h"
#include "device/devcomm.h"
#include "plan.h"

namespace msccl {

class Bootstrap;

constexpr uint64_t kCommMagic = 0x6d7363636c616d64ull;  // "msccl amd"

// Connection key: (group, channel, peer); group = algorithm index, or kRingGroup for the ring
// fallback's channels.  Every group owns its connections (transport.cc).
constexpr int kRingGroup = kMaxAlgos;
constexpr int kTreeGroup = kMaxAlgos + 1;  // the tree fallback's chain connections
constexpr int kFlatGroup = kMaxAlgos + 2;  // the flat tree's all-pairs connections (channel 0)
constexpr int kNumGroups = kMaxAlgos + 3;
struct ConnKey {
  int group, chan, peer;
};

// Per-rank transport table exchanged during init: for every (group, channel, peer) the offsets,
// inside this rank's transport arena, of the receive FIFOs / tail word (this rank receiving
// from peer) and of the head word (this rank sending to peer).  -1 = no connection.
// Sub-connection k of a key sits at base + k * stride.
struct PeerOffsets {
  int64_t recvLL, recvSimple, recvTail, sendHead;
  int64_t llStride, simpleStride, wordStride, pad;
};

// One algorithm (or ring program) on the device: fixed-stride thread-block images and the
// slot-indexed connection records (entry tb * connSplit + sub) of its thread blocks.
struct DevAlgoHost {
  char* dImages = nullptr;
  int tbStride = 0;
  int nBlocks = 0;
  DevSendConn* dSend = nullptr;
  DevRecvConn* dRecv = nullptr;
  int connSplit = 1;
  // this schedule's range of dependency-flag / launch-epoch slots (init.cc: allocSlots): a launch
  // reads and advances only its own schedule's epochs
  int slotBase = 0;
  int slotCount = 0;
};

// A thread block whose exchange with its single peer may run fused (transport.cc: fusableTbs):
// tb index, index of its `s` (the `rrc` follows), channel, peer.
struct FuseCandidate {
  int16_t tb, index, chan, peer;
};
constexpr int kMaxFuse = 64;  // candidates per algorithm exchanged at init

struct ncclCommImpl;
}  // namespace msccl

struct ncclComm {
  uint64_t magic = msccl::kCommMagic;
  int rank = 0, nRanks = 1, cudaDev = 0;
  int64_t busId = 0;
  std::vector<msccl::Algorithm> algos;
  std::vector<msccl::Registration> regs;
  std::vector<msccl::DevAlgoHost> devAlgos;
  // per algorithm: this rank's fold order when the schedule runs as the one-hop fold (lower.cc;
  // empty: it does not) and the fold kernel's program for it (nBlocks 0 when empty)
  struct FoldProgram {
    std::vector<int> chunkClass;            // class of every chunk (lower.h)
    std::vector<std::vector<int>> order;    // this rank's fold order (ranks) per class; empty: not lowered
    // the two-phase form (lower.h: FoldLowering::twoPhase, agreed by every rank at init): the
    // owner of every chunk; empty when the schedule has none
    std::vector<int> owner;
  };
  std::vector<FoldProgram> algoFold;
  // per algorithm: the direct form of a Simple schedule (lower.h: DirectLowering, agreed by every
  // rank at init; coll -1: none) and its device program (directAlgos: the fold orders, RS / AR)
  struct DirectProgram {
    int coll = -1;
    std::vector<int> chunkClass;
    std::vector<std::vector<int>> order;  // this rank's fold order (ranks) per class
  };
  std::vector<DirectProgram> algoDirect;
  std::vector<msccl::DevAlgoHost> directAlgos;
  // the ring fallback's Simple ReduceScatter as a direct form (one class: this rank's ring order
  // r+1, r+2, ..., r, reduce_scatter.h:50-65); its AllGather needs no program
  msccl::DevAlgoHost ringDirectRS;
  // communicators created together by one ncclCommInitAll with every rank on one device share a
  // nonzero clique id: a group call of all of them is one fused launch (the direct form's condition)
  uint64_t clique = 0;
  std::vector<int> algoSet;  // per algorithm: the small kernel's transfer set (transport.cc: algoUpload)
  // per algorithm: thread block b's program is one fused exchange of input chunk src + b * stride
  // into chunk dst + b * stride of buffer dstBuf (the pair kernel, RankWork::pairSrc); src -1: not
  struct PairForm {
    int src = -1, dst = 0, stride = 0, dstBuf = 0;
  };
  std::vector<PairForm> algoPair;
  std::vector<uint8_t> algoPairAll;  // every rank runs the schedule in pair form (init.cc: applySplits)
  std::vector<msccl::DevAlgoHost> foldAlgos;
  msccl::DevAlgoHost ringAlgos[6];  // ring fallback programs, [4] = tree, [5] = flat tree (transport.cc: ringUpload)
  msccl::Knobs knobs;              // environment knobs, read once at init, identical on every rank
  bool ringFallback = true;        // MSCCL_AMD_RING_FALLBACK (default 1), same on every rank
  bool anyRemote = false;          // some peer runs on another GPU (xGMI): no LL128 unless allowed
  std::vector<int> algoSplit;      // workgroups per XML thread block, per algorithm (same on all ranks)
  std::vector<int> algoSplitBase;  // the split of the default budget (algoSplit is wider for 2 co-resident LL ranks)
  std::vector<int> algoMaxBlocks;  // per algorithm: the most thread blocks of any rank's program (same on all ranks)
  std::vector<int> algoSendRun;    // per algorithm: longest run of send chunks before a receive, max over
                                   // every rank's program (same on all ranks)
  std::vector<std::vector<msccl::FuseCandidate>> algoFuse;  // per algorithm: thread blocks running fused
                                                            // (both ends of the exchange agreed at init)
  int maxSplit = 1;                // sub-connections per (channel, peer)
  int coResident = 1;              // ranks of this communicator on this rank's GPU
  std::vector<int> foldClasses;    // per algorithm: algoFold's class count (0: not lowered)
  std::vector<int> foldTwoPhase;   // per algorithm: algoFold has the two-phase form (owner table)
  std::vector<int> directClasses;  // per algorithm: the direct form's fold orders (AG: 1), 0: none
  msccl::PlanContext planCtx;      // what planCall reads (set at the end of init: commFinish)

  // transport
  std::vector<msccl::ConnKey> sendKeys, recvKeys;
  char* arena = nullptr;
  size_t arenaSize = 0;
  std::vector<msccl::PeerOffsets> table;              // [kNumGroups * kMaxChannels * nRanks] own table
  std::vector<char*> peerArena;                        // per rank: mapped arena base
  std::vector<bool> peerArenaIpc;                      // opened through hipIpcOpenMemHandle
  msccl::DevSendConn* ringSend = nullptr;              // ring fallback connections [kRingChannels]
  msccl::DevRecvConn* ringRecv = nullptr;
  msccl::DevSendConn* treeSend = nullptr;              // tree fallback connections [2 * kRingChannels]
  msccl::DevRecvConn* treeRecv = nullptr;
  msccl::DevSendConn* flatSend = nullptr;              // flat tree connections [nRanks][flatSubs] (tb 0 has none)
  msccl::DevRecvConn* flatRecv = nullptr;
  // sub-connections per flat connection: kFlatSubs, or the lowered large calls' workgroups per
  // rank when a schedule runs them (init.cc: applySplits; the same on every rank)
  int flatSubs = msccl::kFlatSubs;
  int llSlotLines = 0, simpleSlotBytes = 0;
  int buffSizes[3] = {0, 0, 0};

  // MSCCL state
  uint64_t* dFlags = nullptr;            // [slotTotal][kFlagStride] flags, then [slotTotal] epochs
  int slotTotal = 0;
  msccl::TraceEvent* dTrace = nullptr;   // MSCCL_AMD_TRACE: [216 * maxSplit][traceEvents]
  int traceEvents = 0;
  bool traceLight = false;               // MSCCL_AMD_TRACE=2: start / end per workgroup, small kernel kept
  msccl::NpkitLog* dNpkit = nullptr;      // MSCCL_AMD_NPKIT (npkit.cc)
  msccl::NpkitEvent* dNpkitEvents = nullptr;
  uint64_t* dNpkitHeads = nullptr;
  int npkitCap = 0, npkitClockKHz = 0;
  void* scratch = nullptr;
  size_t scratchSize = 0;
  uint32_t workIndex = 1;    // host launch counter (the device epoch drives the flags)
  msccl::DevComm* dComm = nullptr;

  // failure handling
  uint32_t* hostAbort = nullptr;   // mapped
  uint32_t* hostErr = nullptr;     // mapped
  uint32_t* devAbort = nullptr;
  uint32_t* devErr = nullptr;
  double timeoutSec = 0.0;         // MSCCL_AMD_TIMEOUT_SEC: bound on a single device wait (0 = none)
  uint64_t timeoutTicks = 0;       // the same in s_memrealtime ticks (100 MHz)
  uint32_t llFlagMask = 0xffffffffu, llCleanMask = 0x7ffffff8u;  // MSCCL_AMD_TEST_LL_CLEANUP
  ncclResult_t asyncError = ncclSuccess;

  // rendezvous
  msccl::Bootstrap* boot = nullptr;
  bool ownsBoot = false;

  // what the most recent collective ran (introspection: mscclAmdCommInfo "last")
  struct LastLaunch {
    int algo = -2, proto = -1, split = 0, merge = 0, ringColl = 0, ringChannels = 0, blocks = 0, small = 0;
    int set = 0;  // the small kernel's transfer set (devcomm.h: kSetAll / kSetExchange)
    int pair = 0;  // the exchange ran in the pair kernel (mscclPairKernel)
    int kernel = -1;  // 0 mscclKernel, 1 mscclSmallKernel, 2 mscclFoldKernel, 3 mscclPairKernel, 4 mscclTwoPhaseKernel,
                      // 5 mscclDirectKernel
  } last;

  // user reduction ops (ncclRedOpCreatePreMulSum, enqueue.cc:1529-1580): a free list as in the
  // reference; op ids are ncclNumOps + index, mangled with the communicator (comm.h:223-235)
  struct UserRedOp {
    int freeNext = -1;      // -1 = allocated
    ncclDataType_t datatype = ncclFloat32;
    uint64_t scalarArg = 0; // scale bits (host immediate) or the scale's device address
    bool argIsPtr = false;
  };
  std::vector<UserRedOp> userRedOps;
  int userRedOpFreeHead = 0;

  hipStream_t userStream = nullptr;
  bool userStreamSet = false;
  hipEvent_t doneEvent = nullptr;
  std::string lastError;
};

namespace msccl {

// init.cc
ncclResult_t commSetupTransport(std::vector<ncclComm*>& comms, Bootstrap* boot);
ncclResult_t commFree(ncclComm* comm, bool peerBarrier);
bool commValid(const ncclComm* comm);

// npkit.cc
ncclResult_t npkitSetup(ncclComm* comm);
ncclResult_t npkitDump(ncclComm* comm, const char* dir);  // dir null: $NPKIT_DUMP_DIR or /tmp/
void npkitFree(ncclComm* comm);

// transport.cc
size_t tableIndex(int group, int chan, int peer, int nRanks);
ncclResult_t transportPlan(ncclComm* comm);                 // keys, arena layout, allocation, own table
ncclResult_t transportConnect(ncclComm* comm, const std::vector<std::vector<PeerOffsets>>& tables,
                              const std::vector<char*>& peerBases, const std::vector<int>& peerRemote);
ncclResult_t algoUpload(ncclComm* comm);
int algoSendRunOf(const Algorithm& a);
std::vector<FuseCandidate> fusableTbs(const Algorithm& a);
// The pair form of a schedule whose exchanges run fused as `fused` lists them (transport.cc), or
// src -1.  A schedule in pair form on every rank with the pair kernel on everywhere is not lowered
// by default (init.cc: applySplits): the pair kernel's fixed cost is the fold's or less.
ncclComm::PairForm pairFormOf(const Algorithm& a, const std::vector<FuseCandidate>& fused);
bool sendCopyFusable(const Algorithm& a, const std::vector<Transfer>& ts, size_t i);
ncclResult_t ringUpload(ncclComm* comm);
bool flatEnabled(const ncclComm* comm);  // the flat tree's connections and program exist

// enqueue.cc
int typeSize(ncclDataType_t t);

}  // namespace msccl

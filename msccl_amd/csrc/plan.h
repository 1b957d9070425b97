// MSCCL algorithm selection + per-call chunk math (pure host functions, no GPU).
//
//   ArgsCheck                     misc/argcheck.cc:36-80
//   in-place / totalCount         graph/tuning.cc:312-342
//   algorithm match               graph/tuning.cc:344-382 (+ NCCL_ALGO / NCCL_PROTO gates, 185-218)
//   thread counts                 graph/tuning.cc:14-32,78-85; enqueue.cc:486-523
//   chunk math / maxAllowedCount  enqueue.cc:591-734; scratch check enqueue.cc:580-589
//   interpreter chunk parameters  collectives/device/msccl_interpreter.h:79-113
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "algo.h"

namespace msccl {

struct CallDesc {
  int coll;          // Coll
  size_t count;      // user count (recvcount for RS, sendcount for AG)
  int dtype;         // ncclDataType_t
  int redop;         // ncclRedOp_t
  int nRanks, rank;
  bool inPlace;
  int customAlgo = -1;  // ncclCustomCollective algorithm index
  bool remote = false;  // some peer runs on another GPU (ncclComm::anyRemote): link-model defaults
};

struct Plan {
  int algoIndex = -1;
  int proto = 0;
  int refNthreads = 0;
  int64_t count = 0;        // interpreter count (bytes for AllGather/AllToAll)
  int dtype = 0;            // interpreter element type
  int sizeMultiplier = 1;
  int64_t nBytes = 0;
  int maxAllowedCount = 0;
  int nchunksPerLoop = 0;
  int64_t sizePerChunk = 0; // elements per MSCCL chunk
  int64_t chunkSize = 0;    // elements per interpreter iteration
  int64_t minChunk = 0;     // LL: nthreads*8/ts; Simple: (nthreads-32)*8/ts
  size_t scratchNeeded = 0;
  int nIters = 0;
  // ring / tree fallback (algoIndex == -1): kRingAllReduce / kRingReduceScatter / kRingAllGather /
  // kTreeAllReduce (chunkSize is then the final per-channel chunk of the tree loop)
  int ringColl = 0;
  int ringChannels = 0;
  int64_t ringLastChunk = 0;  // LL ReduceScatter / AllGather lastChunkSize (elements)
  // ringColl == kTreeFlat: the collective the fold kernel runs (kRingAllReduce for the flat tree,
  // kRingReduceScatter / kRingAllGather for the flat forms of the ring's)
  int flatColl = 0;
  // a lowered schedule with several fold orders (lowerToFoldPlan): 16-B packs per chunk, else 0
  int64_t foldChunkPacks = 0;
  // a lowered schedule's kernel (lowerToFoldPlan): kLowerFold, or for calls above the fold's
  // limit kLowerPair (2 ranks) / kLowerTwoPhase
  int lowerMode = 0;
  // the call may run the schedule's direct form (planCall: directEligible) if every rank of the
  // communicator is in its launch (enqueue.cc: launchGroup decides); the plan is otherwise the
  // schedule's own.  directChunkPacks: 16-B packs per output chunk for the class lookup (0: one class)
  bool directOk = false;
  int64_t directChunkPacks = 0;
};
enum : int { kLowerFold = 0, kLowerPair = 1, kLowerTwoPhase = 2 };
// 16-B packs per FIFO step of the two-phase fold (a slot holds 2048 at the default LL FIFO)
constexpr int64_t kTwoPhaseStepPacks = 1024;

// Every environment knob the per-call planning reads, captured once at communicator init
// (NCCL_PARAM caches its getenv the same way, include/param.h:99-108).  All ranks must plan
// identical launch geometry, so init also checks that every rank captured the same values
// (init.cc: the SplitRecord allgather).  Plain data: compared with memcmp.
struct Knobs {
  int32_t mscclOn;           // NCCL_ALGO enables MSCCL (tuning.cc:186,217; on unless excluded here)
  int32_t protoOn[3];        // NCCL_PROTO gates per protocol (tuning.cc:188-197)
  int32_t nthreads;          // NCCL_NTHREADS (-2 = unset, tuning.cc:12)
  int32_t ll128Nthreads;     // NCCL_LL128_NTHREADS (tuning.cc:13)
  int64_t buffSizes[3];      // NCCL_LL_BUFFSIZE / NCCL_LL128_BUFFSIZE / NCCL_BUFFSIZE (init.cc:455-472)
  int32_t ringChannels;      // MSCCL_AMD_RING_CHANNELS (0 = auto)
  int32_t split;             // MSCCL_AMD_SPLIT (0 = auto)
  int32_t targetWgs;         // MSCCL_AMD_TARGET_WGS (0: by protocol, chooseSplit)
  int32_t merge;             // MSCCL_AMD_MERGE (0 = as many as fit)
  int32_t ringFallback;      // MSCCL_AMD_RING_FALLBACK
  int32_t ll128Remote;       // MSCCL_AMD_LL128_REMOTE: allow LL128 towards peers on other GPUs
  int32_t ringOn, treeOn;    // NCCL_ALGO enables Ring / Tree for the fallback (tuning.cc:188-197)
  int64_t treeMaxBytes;      // MSCCL_AMD_TREE_MAX_BYTES: AllReduce fallback calls up to this size take the
                             // tree (-1: 512 KiB for the flat tree, else 16 KiB per rank); when set it also
                             // caps a rank's block for the flat ReduceScatter / AllGather
  int32_t smallKernel;       // MSCCL_AMD_SMALL_KERNEL: one-iteration LL launches take mscclSmallKernel
  int32_t referenceSelection;  // MSCCL_AMD_REFERENCE_SELECTION: the reference's MSCCL gating (below)
  int32_t fuse;              // MSCCL_AMD_FUSE: fused s + rrc exchanges (transport.cc: fusableTbs)
  int32_t treeFlat;          // MSCCL_AMD_TREE_FLAT: the tree's values in one hop (plan.cc: makeFlatTreePlan)
  int32_t lower;             // MSCCL_AMD_LOWER: one-hop AllReduce schedules run as the fold (lower.cc)
  int32_t simpleBuffEnv;     // NCCL_BUFFSIZE was set (else a communicator of one GPU takes kLocalSimpleBuff)
  int64_t lowerMaxBytes;     // MSCCL_AMD_LOWER_MAX_BYTES: largest call (bytes per rank) lowered (-1: by ranks)
  int32_t pairKernel;        // MSCCL_AMD_PAIR_KERNEL: pair-form exchanges take mscclPairKernel (rank-local)
  int32_t lowerLarge;        // MSCCL_AMD_LOWER_LARGE: lowered calls above the fold's limit run lowered too
                             // (2 ranks: the pair kernel; more: the two-phase fold; plan.cc: lowerLargePlan)
  int32_t forceRemote;       // MSCCL_AMD_FORCE_REMOTE: every peer treated as on another GPU (a test knob)
  int32_t twoPhaseStep;      // MSCCL_AMD_TWO_PHASE_STEP: 16-B packs per FIFO step of the two-phase fold (0: default)
  int32_t direct;            // MSCCL_AMD_DIRECT: Simple schedules' direct form when every rank is in one launch
  static Knobs fromEnv();
};

// The Simple FIFO of a communicator whose ranks all share one GPU, unless NCCL_BUFFSIZE is set:
// 256 KiB (eight 32-KiB slots) instead of the reference's 4 MiB.  Every FIFO hand-off then stays
// in the L2 / MALL, and a ring's per-step skew costs 32-KiB steps: the 8-rank C4 ring 2.07 ->
// 1.47 ms, C5 and the 2-rank shapes 3-25 % faster (profiles/r04i_c4knobs.txt, r04j_c4knobs.txt;
// 128 and 64 KiB lose again).  Connections between GPUs keep the reference's size, and so does a
// communicator with a Simple schedule that sends more than two chunks before it receives
// (init.cc: applySplits).
constexpr int64_t kLocalSimpleBuff = 256 << 10;
// init's decision (init.cc: applySplits), the same on every rank: oneGpu = every rank of the
// communicator on one GPU; sendRun = per algorithm the longest run of sent chunks before a
// receive over every rank's program (algoSendRunOf)
bool useLocalSimpleFifo(bool oneGpu, const Knobs& k, const std::vector<Algorithm>& algos,
                        const std::vector<int>& sendRun);

int refTypeSize(int dtype);
bool inPlaceOf(int coll, const void* send, const void* recv, size_t count, int dtype, int rank);
// Returns the selected algorithm index or -1 (the reference falls back to ring/tree there).
int selectAlgo(const std::vector<Algorithm>& algos, const std::vector<Registration>& regs, const CallDesc& c,
               const Knobs& k);
// Fills *p; returns an ncclResult_t code.
int makePlan(const std::vector<Algorithm>& algos, int algoIndex, int protoOverride, const CallDesc& c, const Knobs& k,
             Plan* p);
// Workgroups per XML thread block for an algorithm (protocol proto) whose largest rank program
// has maxBlocks thread blocks when coResident ranks share a GPU: the largest power of two <=
// kMaxSplit that keeps the GPU's workgroups within MSCCL_AMD_TARGET_WGS (default by protocol: 256
// = one per CU for LL / LL128, 512 for Simple).  MSCCL_AMD_SPLIT forces a value.  Every rank must
// compute the same value.  wide: the budget of two co-resident ranks' LL schedules, 512 (for large
// calls; makeWork steps a call back towards the default split while a workgroup would move less
// than kWideSplitMinBytes).
int chooseSplit(int maxBlocks, int coResident, const Knobs& k, int proto, bool wide = false);
// Two co-resident ranks, graph replay, same box (profiles/r05w_target_wgs.txt): the 2-rank two-phase
// all-pairs x16 at 512 workgroups per GPU against 256: 4 MiB 25.5 against 23.1 us (16 KiB per
// workgroup), 8 MiB 31.0 against 33.2, 16 MiB 46.5 against 52.5, 32 MiB 79.7 against 102.8.
constexpr int64_t kWideSplitMinBytes = 32 << 10;
// The reference's fallback when no MSCCL algorithm matches (enqueue.cc:461-476): a ring
// AllReduce / ReduceScatter / AllGather (collectives/device/all_reduce.h:14-100,
// reduce_scatter.h:13-67, all_gather.h:13-78).  Fills *p (algoIndex -1, ringColl set) and returns
// 0, or returns ncclInvalidUsage when the collective / op has no ring (AllToAll, custom, Avg).
// Channels, protocol and thread count are this build's choice (oracle/ring.py: ring_params).
int makeRingPlan(const CallDesc& c, const Knobs& k, Plan* p);
// The flat forms (kTreeFlat, run by mscclFoldKernel, interpreter.h: runFold), one hop each:
//   a tree AllReduce plan (makeRingPlan chose the tree, LL, op Sum..Min, 2..16 ranks): every rank
//   sends its input to every peer and folds the n inputs in the chain tree's order x_{n-1} (+)
//   x_{n-2} (+) ... (+) x_0, instead of 2 (n - 1) hops;
//   an LL ring ReduceScatter (op Sum..Min) or AllGather (the whole LL range, 512 KiB in all, by
//   default; MSCCL_AMD_TREE_MAX_BYTES, when set, also caps a rank's block): every rank sends block
//   p to peer p and folds its own block in
//   the ring's order x_{r+1} (+) x_{r+2} (+) ... (+) x_{r+n-1} (+) x_r (ReduceScatter), or sends
//   its block to every peer and stores each peer's at its place (AllGather), instead of n - 1.
// Returns 0, or nonzero when the call does not qualify (the plan is then unchanged).
int makeFlatTreePlan(const CallDesc& c, const Knobs& k, Plan* p);
// A call of an MSCCL AllReduce schedule that lower.cc proved to be a one-hop fold (LL, op
// Sum..Min, at most MSCCL_AMD_LOWER_MAX_BYTES per rank): turns the schedule's plan into the fold
// kernel's (ringColl kTreeFlat, flatColl kRingAllReduce; algoIndex kept: the fold runs with the
// schedule's own fold order, ncclComm::foldAlgos).  Returns 0, or nonzero (plan unchanged).
// classes: the schedule's fold orders (lower.h); with several, the call's chunks must be whole
// 16-B packs (each pack folds in its chunk's order).
// Calls above that limit (MSCCL_AMD_LOWER_LARGE, default on) run lowered as well, with the
// schedule's values and without its scratch: 2 ranks as the pair exchange (each rank sends its
// input, folds the peer's copy into its own: one hop, 6 S HBM bytes per rank against the two-phase
// all-pairs' 7.5 S), more ranks as the two-phase fold when the schedule has that form
// (twoPhase: lower.h) and its chunks are whole packs (9 S against the scratch form's 11.6 S at 8
// ranks).  Otherwise nonzero: the interpreter runs the schedule.
int lowerToFoldPlan(const CallDesc& c, const Knobs& k, int classes, bool twoPhase, Plan* p);
// What a communicator's per-call planning reads besides the call itself (enqueue.cc: planOp).
// The introspection mscclAmdLaunchPlanJson fills the same from XML files and a placement, so
// what it reports is what a communicator of that placement launches.
struct PlanContext {
  const std::vector<Algorithm>* algos = nullptr;
  const std::vector<Registration>* regs = nullptr;
  const Knobs* knobs = nullptr;                   // after init's agreed adjustments (FIFO sizes)
  const std::vector<int>* foldClasses = nullptr;  // per algorithm: fold orders when lowered, else 0
  const std::vector<int>* foldTwoPhase = nullptr; // per algorithm: the lowering has a two-phase form
  const std::vector<int>* directClasses = nullptr; // per algorithm: the direct form's fold orders, 0: none
  bool oneLaunch = false;     // the communicator's group calls are one fused launch (ncclComm::clique)
  bool ringDirect = false;    // oneLaunch, MSCCL_AMD_DIRECT and no trace / NPKit: the ring fallback's
                              // Simple ReduceScatter / AllGather may run as the direct form
  bool flat = false;          // the flat group's connections exist (transport.cc: flatEnabled)
  bool ringFallback = true;   // MSCCL_AMD_RING_FALLBACK
  size_t scratchSize = 0;     // MSCCL scratch allocated at init
};
// One call of a communicator of more than one rank (the reference's selection, enqueue.cc:448-476
// and 591-734): an MSCCL schedule (LL128 run as LL towards other GPUs unless allowed), the
// lowered fold, or the ring / tree / flat fallback.  asyncMany: the group holds more than one op
// of the communicator.  Returns an ncclResult_t code.
int planCall(const PlanContext& ctx, const CallDesc& c, bool asyncMany, Plan* p);
// The default of MSCCL_AMD_LOWER_MAX_BYTES:the largest call (bytes per rank) a lowered schedule
// runs as the fold.  Ranks sharing one GPU: measured (4 KiB for 2 ranks, 128 KiB above).  Peers
// on other GPUs: the xGMI link model below, capped at the fold kernel's own
// throughput limit.
int64_t defaultLowerMaxBytes(int nRanks, bool remote);
// The link model's crossover (bytes per rank) between the fold and the two-phase all-pairs
// schedule of n ranks, one rank per GPU: the fold sends f.S on each of its n - 1 links in one
// hop, the two-phase schedule 2 f.S / n per link in two hops and with the interpreter's larger
// fixed cost, so the fold wins while S < (dF + L) B / (f (1 - 2/n)).  Infinite (-1) for n <= 2,
// where both move the same link bytes in one hop.
int64_t foldLinkCrossoverBytes(int nRanks);
// the model's parameters
constexpr double kXgmiLinkOneWayGBs = 76.8;  // MI355X: 153.6 GB/s per link, both directions
constexpr double kXgmiHopUs = 2.0;           // one cross-GPU LL hand-off (assumed until the 8-GPU sweep)
constexpr double kInterpFixedUs = 5.0;       // interpreter over fold fixed cost (8 ranks, 128 B: 13.8 - 8.8 us)
constexpr int64_t kFoldMaxBytesCap = 256 << 10;  // co-resident even point of the fold (16 workgroups)

}  // namespace msccl

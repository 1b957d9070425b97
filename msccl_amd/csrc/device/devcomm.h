// Device-visible data model of the MI355X MSCCL runtime (shared by host C++ and HIP kernels).
//
// Replaces the reference's ncclDevComm / ncclConnInfo / mscclThreadBlock device copies
// (include/devcomm.h:83-295, include/msccl.h:46-118).  Differences by design:
//   * the per-tb program is a packed blob (16-B transfers + int16 dep/reduction tables)
//     copied into LDS by each workgroup, instead of a fixed 5,904-B mscclThreadBlock;
//   * one connection = receiver-owned FIFO in uncached (fine-grained) HBM plus a head word in
//     the sender's memory and a tail word in the receiver's memory; the sender writes the
//     FIFO over xGMI (peer pointer or hipIpc mapping);
//   * a launch may carry the work of several co-resident ranks (ranks that share one GPU):
//     RankWork[i] owns blocks [blockBase, blockBase + nBlocks);
//   * one XML thread block may run as `split` workgroups: workgroup k of a tb owns the k-th
//     1/split of the 16-B packs of every MSCCL chunk (by position inside the chunk) and its own
//     sub-connection (FIFO, head/tail words, step counter) and dependency flag, so the values
//     produced are the same as with one workgroup (the split is by element, every element
//     keeps its operations and their order).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace msccl {

constexpr int kFifoSteps = 8;          // NCCL_STEPS: Simple FIFO slots per sub-connection
// LL / LL128 FIFO slots per sub-connection (the same 8 as the reference's NCCL_STEPS).
// Calls may be merged here (full iterations, a transfer's chunks), which the reference never
// does.  What a merged call must not break is that a thread block's sends issued before its next
// receive fit its FIFO (both ends of a pair may send first).  The host bounds every run of
// consecutive sends of a schedule to kMaxRunSlots slots per sub-connection: half the FIFO, so
// one launch iteration's run can also sit behind the previous one unconsumed.
constexpr int kLLFifoSlots = kFifoSteps;
constexpr int kMaxRunSlots = 4;
constexpr int kMaxLaunchRanks = 16;    // ranks fused into one launch (same device, same group)
constexpr int kFlagStride = 4;         // uint64 words per flag (32 B, mscclFlag padding)
constexpr int kMaxSplit = 8;           // workgroups per XML thread block (sub-connections)
constexpr int kNT = 512;               // threads per workgroup (8 waves of 64)
constexpr int kMaxFoldPeers = 15;      // flat tree fold: peers of one rank (MSCCL_MAX_REDUCE_FUSION 16 ranks)
// flat tree: sub-connections per peer = most fold workgroups per rank.  16: one 16-B pack per
// lane up to 128 KiB (fp16 / bf16) per rank; with 4, a 128-KiB 8-rank fold took 23.3 us against
// 12.5 (lanes walking 4 packs, each poll waiting for the last), 64 KiB 15.6 against 11.3, small
// calls unchanged (profiles/r04t_lat.txt).  LL FIFOs only: 8 MiB per peer
constexpr int kFlatSubs = 16;
// Lowered large calls (the pair kernel on the flat connections for 2 ranks, the two-phase fold
// for more: lower.h) run up to this many workgroups per rank, one sub-connection each (the
// workgroup count travels in RankWork::split, a byte)
constexpr int kMaxFlatSubs = 128;
constexpr int kFoldPacksPerWg = 512;   // flat tree: a fold workgroup per 512 packs (8 KiB) of the call
constexpr int kMaxFoldClasses = 16;    // lowered schedules (lower.cc): fold orders per schedule
constexpr int kMaxFoldChunks = 1024;   // lowered schedules with several orders: chunks per loop
constexpr int kMaxDirectClasses = 256; // the direct form (DirectLowering): fold orders (a 32-ring schedule: 256)

// Device trace event (mscclAmdTraceRead).
struct TraceEvent {
  uint64_t ts;
  uint16_t type, step;
  uint32_t arg;
};
enum TraceType : uint16_t {
  kEvSetup = 1,      // program staged, connections read
  kEvDepWait = 2,    // dependency flags satisfied (step = transfer index)
  kEvPrimBegin = 3,  // arg = transfer type << 24 | elements of this workgroup (capped)
  kEvPrimEnd = 4,    // arg = 10-ns ticks waited for the Simple tail << 16 | ticks waited for send credit
  kEvEnd = 5,        // workgroup done
  kEvHeader = 0xFFFF
};

// NPKit-compatible event log (include/msccl_amd_npkit.h): 16-B events {type:8 | size:32 |
// rsvd:24, timestamp} (npkit_struct.h:8-17), one buffer per thread block, kept across launches.
struct NpkitEvent {
  uint64_t bits;  // type | size << 8 | rsvd << 40
  uint64_t ts;
};
struct NpkitLog {
  NpkitEvent* events;    // [kNpkitDevBuffers][cap]
  uint64_t* heads;       // [kNpkitDevBuffers] events written so far (may exceed cap: the rest dropped)
  int64_t cpuOffsetNs;   // host system_clock ns = npkitTicksToNs(GPU clock ticks, clockKHz) + cpuOffsetNs
  int32_t cap;
  int32_t clockKHz;      // s_memrealtime rate (100000 kHz on MI355X)
};
// GPU clock ticks -> ns for a clock of khz kHz, exact for any rate (no rounded period: a 3.33-ns
// period taken as 3 ns would drift linearly) and free of overflow for any uptime.
__host__ __device__ inline int64_t npkitTicksToNs(uint64_t ticks, int32_t khz) {
  const uint64_t k = (uint64_t)khz;
  return (int64_t)((ticks / k) * 1000000ull + (ticks % k) * 1000000ull / k);
}
constexpr int kNpkitDevBuffers = 216;  // MSCCL_MAX_NUM_THREAD_BLOCKS: buffer = thread block

// LL FIFO line (ncclLLFifoLine, devcomm.h:35-48): two 8-B {4-B data, 4-B flag} granules.
struct alignas(16) LLLine { uint32_t d0, f0, d1, f1; };

// Packed transfer (mscclTransfer, msccl.h:46-58).
struct alignas(16) DevTransfer {
  int16_t srcoff, dstoff;
  uint8_t srcbuf, dstbuf, type, count;
  int16_t depPtr, numDeps;
  int16_t redPtr;
  uint8_t numReds, hasDep;
};
static_assert(sizeof(DevTransfer) == 16, "DevTransfer must be 16 bytes");

// First 16 B of a thread-block image.  Image = [DevTbHeader][nsteps DevTransfer][ndeps int16
// dependency tb][ndeps int16 dependency step][nreds int16 reduction source offset], padded to
// 16 B; a group's images have one stride (RankWork::tbStride), so workgroup b finds image b
// without first reading a table (one memory round trip in the kernel prologue).
struct alignas(16) DevTbHeader {
  int16_t hasSend, hasRecv;     // the tb's connection records (RankWork::send / ::recv) are in use
  uint16_t nsteps, ndeps;
  uint16_t nreds, pad;
  uint32_t reserved;
};
constexpr int kMaxImage16 = 1 + 256 + (3 * 256 * 2 + 15) / 16;  // largest image in 16-B units
static_assert(sizeof(DevTbHeader) == 16, "DevTbHeader must be 16 bytes");

struct DevSendConn {
  LLLine* ll;                  // receiver's LL FIFO (peer memory)  [kLLFifoSlots][llSlotLines]
  char* simple;                 // receiver's Simple FIFO (peer memory) [kFifoSteps][simpleSlotBytes]
  uint64_t* remoteTail;         // receiver's tail word (peer memory)
  uint64_t* head;               // my head word, written by the receiver
  uint64_t step;                // persistent step counter (owned by one workgroup)
  uint64_t headSeen;            // last head value read: credit known without a poll while step < headSeen + 8
  int32_t llSlotLines;
  int32_t simpleSlotBytes;
  int32_t remote;               // 1: receiver on another GPU (system-scope release before a tail post);
                                // 2: local, agent fences (MSCCL_AMD_SIMPLE_FENCE); 0: local, sc0 sc1 form
  int32_t pad;
};

struct DevRecvConn {
  LLLine* ll;                  // my LL FIFO
  char* simple;                 // my Simple FIFO
  uint64_t* tail;               // my tail word, written by the sender
  uint64_t* remoteHead;         // sender's head word (peer memory)
  uint64_t step;
  uint64_t tailSeen;            // last Simple tail value read (data known present below it)
  int32_t llSlotLines;
  int32_t simpleSlotBytes;
  int32_t remote;               // 1: sender on another GPU (system-scope acquire after a tail is seen);
                                // 2: local, agent fences (MSCCL_AMD_SIMPLE_FENCE); 0: local, sc0 sc1 form
  int32_t pad;
};
static_assert(sizeof(DevSendConn) == 64 && sizeof(DevRecvConn) == 64, "connection records are four 16-B units");

struct DevComm {
  uint64_t* flags;              // [slots][kFlagStride]: every schedule's range (ncclComm::slotTotal)
  volatile uint32_t* abortFlag; // host-mapped
  uint32_t* errWord;            // host-mapped: 0 ok, else error code (1 timeout, 2 bad program)
  uint64_t timeoutTicks;        // s_memrealtime ticks (100 MHz) a single wait may last; 0 = for ever
  int32_t maxSplit;             // sub-connections per (channel, peer): conn k of key c = send[c*maxSplit+k]
  int32_t pad;
  // Launch epoch (the reference's host-side workIndex, enqueue.cc:714-721, kept on the device so
  // that a captured hipGraph replays correctly), one word per workgroup slot of every schedule
  // (slot = tb * maxSplit + sub within the schedule's range, the flag index): a workgroup reads
  // its own slot at start and writes slot + 1 at its end, together with the slots of its schedule
  // this launch does not run (subs beyond its split, ring channels beyond its count).  Every slot
  // of a schedule therefore holds the same value at each of its launch starts, no counter is
  // shared by the workgroups of a launch (a contended "last one out" counter cost several us per
  // launch at 512 workgroups), and a launch writes no other schedule's words.
  uint64_t* epochs;             // [slots]
  uint64_t* unused;
  // NPKit-style trace (null = off): [slot = tb * maxSplit + sub][traceEvents]
  struct TraceEvent* trace;
  int32_t traceEvents;
  int32_t pad2;
  // LL / LL128 flag arithmetic (devcomm.h:56-63): flag = (step + 1) & llFlagMask, and a sender
  // stamps the unused lines of a slot on steps with (step & llCleanMask) == llCleanMask.
  // Production: 0xffffffff / 0x7ffffff8.  MSCCL_AMD_TEST_LL_CLEANUP=1 is the reference's
  // TEST_LL_CLEANUP build (NCCL_LL_FLAG_MAX 0x100, NCCL_LL_CLEAN_MASK 0x078): the flag wraps every
  // 256 steps and the cleanup runs 8 steps in every 128, so tests reach it in a few launches.
  uint32_t llFlagMask;
  uint32_t llCleanMask;
};

// Ring fallback kinds (RankWork::ringColl)
// Ring / tree fallback kinds (RankWork::ringColl).  kTreeAllReduce: the reference's tree
// AllReduce (all_reduce.h:103-298) on a chain, two thread blocks per channel (reduce up /
// broadcast down, as runTreeSplit), offsets gridOffset + channel * chunkSize.
// kTreeFlat is a host-side plan kind only: the flat tree runs as an MSCCL schedule (ringColl 0 in
// its RankWork, plan.cc: makeFlatTreePlan).
enum : int { kRingNone = 0, kRingAllReduce = 1, kRingReduceScatter = 2, kRingAllGather = 3, kTreeAllReduce = 4,
             kTreeFlat = 5 };

// One rank's share of a launch (the reference passes ncclDevComm* + a 64-B ncclWorkElem,
// common.h:263-266; here the whole descriptor rides in the kernel argument block).
struct RankWork {
  const void* sendbuff;
  void* recvbuff;
  void* scratch;
  DevComm* comm;
  // copies of the DevComm fields every workgroup needs at start (kernel arguments: no
  // dependent global load before the first connection / epoch load)
  DevSendConn* send;
  DevRecvConn* recv;
  uint64_t* flags;
  uint64_t* epochs;
  int32_t maxSplit;
  int32_t foldPacksPerWg;       // fold kernel: packs per workgroup, floor(packs / split) (no division on the device)
  const char* images;           // thread-block images, tbStride bytes each
  int32_t tbStride;
  int32_t connSplit;            // connection record of (tb, sub): send / recv [tb * connSplit + sub]
  int64_t sizePerChunk;         // sizePerMscclChunk = count*sizeMultiplier/nchunksPerLoop (elements)
  int64_t chunkSize;            // interpreter chunkSize (elements)
  int64_t minChunk;             // LL: nthreads*8/sizeof(T); Simple: rounding unit (nthreads-32)*8/sizeof(T)
  uint32_t launchSeq;            // host launch counter (diagnostics only; flags use DevComm::epoch)
  int16_t blockBase;
  int16_t nBlocks;              // workgroups = XML thread blocks x split
  int16_t refNthreads;          // reference nthreads (small-reduce switch, chunk rounding)
  uint8_t maxAllowedCount;
  uint8_t split;                // workgroups per XML thread block; each owns 1/split of every op
  uint8_t merge;                // full interpreter iterations run as one (same per-element operations)
  uint8_t foldPeers;            // flat tree (mscclFoldKernel): peers, on the records of thread blocks 1..foldPeers
  int16_t epochSlots;           // the schedule's flag / epoch slots (flags and epochs point at its range)
  // the pair kernel (mscclPairKernel; transport.cc: algoUpload's pair form): thread block b runs
  // one fused exchange of input chunk pairSrc + b * pairStride into chunk pairDst + b * pairStride
  // of buffer pairDstBuf (0 input, 1 output); pairSrc -1: the schedule is not of that form
  int16_t pairSrc, pairDst, pairStride;
  uint8_t pairDstBuf;
  int64_t maxOpElems;           // largest run of sends before a receive (elements, all sub-connections)
  // ring fallback (kRingNone for MSCCL schedules): the program's offsets are chunk / rank indices
  // of the reference's runRing (all_reduce.h:14-100, reduce_scatter.h:13-67, all_gather.h:13-78)
  uint8_t ringColl;
  int16_t ringRanks;
  int32_t foldChunkPacks;       // a lowered schedule folding chunks in several orders: packs per chunk (else 0)
  int64_t ringSize;             // elements of one rank's block (args->count)
  int64_t ringLastChunk;        // LL ReduceScatter / AllGather lastChunkSize (enqueue.cc:653-658)
  // copies of per-communicator constants (kernel arguments: no dependent DevComm load)
  uint64_t timeoutTicks;
  uint32_t llFlagMask, llCleanMask;
  struct TraceEvent* trace;
  int32_t traceEvents;
  int32_t redOpArgIsPtr;        // redOpArg is a device address of the scalar (ncclScalarDevice)
  uint64_t redOpArg;            // PreMulSum scale bits / SumPostDiv divisor (ncclDevRedOpFull::scalarArg)
  NpkitLog* npkit;              // MSCCL_AMD_NPKIT (null = off)
  // the two-phase fold (mscclTwoPhaseKernel): the 16-B packs each rank owns (chunks per rank x
  // foldChunkPacks), and the division by foldChunkPacks as a multiply-high and two shifts (exact
  // for every 32-bit dividend: divMagic of Granlund and Montgomery, computed by the host)
  uint32_t tpOwnedPacks;
  uint32_t tpMagic;
  uint8_t tpSh1, tpSh2;
  uint16_t tpStepPacks;         // packs per FIFO step (at most a slot's): the FIFO footprint in flight
  int16_t directRank;           // the direct form (mscclDirectKernel): this work's rank (the launch holds every rank)
#ifdef MSCCL_RANKWORK_TEST_PAD
  // a deliberate layout split (tools/varbuild.sh's guard test): a kernel object built with this
  // define has a larger RankWork, so it reads every rank's entry after the first of the launch
  // argument block (LaunchArgsN::w) at another offset than the host wrote it
  int32_t testPad;
#endif
};

// Layout stamp of RankWork: every kernel object records the one it was compiled with (kernels.h)
// and communicator setup refuses a library whose objects disagree with the host's
// (dispatch.cc: kernelLayoutMismatch) -- a kernel object left over from before a RankWork change
// reads its arguments at the wrong offsets, an illegal memory access rather than an error code.
// The stamp folds the size and the offsets of fields spread over the whole struct, so a field added,
// removed or resized anywhere (a -D flag given to one object only, a stale object) changes it.
constexpr uint32_t layoutMix(uint32_t h, uint32_t v) { return (h ^ v) * 16777619u; }  // FNV-1a step
constexpr uint32_t kWorkLayout =
    layoutMix(layoutMix(layoutMix(layoutMix(layoutMix(layoutMix(layoutMix(layoutMix(layoutMix(2166136261u,
    (uint32_t)sizeof(RankWork)), (uint32_t)offsetof(RankWork, tbStride)), (uint32_t)offsetof(RankWork, sizePerChunk)),
    (uint32_t)offsetof(RankWork, blockBase)), (uint32_t)offsetof(RankWork, pairSrc)), (uint32_t)offsetof(RankWork, maxOpElems)),
    (uint32_t)offsetof(RankWork, ringSize)), (uint32_t)offsetof(RankWork, npkit)), (uint32_t)offsetof(RankWork, tpStepPacks));

template <int R>
struct LaunchArgsN {
  int32_t nRanks;
  int32_t pad;
  RankWork w[R];
};
using LaunchArgs = LaunchArgsN<kMaxLaunchRanks>;
// A launch of at most two ranks (one rank per process, or the 2-rank co-resident C2 launch) takes
// a kernel whose argument block holds two RankWorks (424 B instead of 3.3 KiB): the HIP runtime
// copies the whole block per launch, about 0.9 us more for the larger one (tools/host_lat).
constexpr int kCompactLaunchRanks = 2;

// Transfer-type sets of the small-call kernel (mscclSmallKernel<..., SET>).  A launch's code is
// fetched into the instruction cache anew by every workgroup's CU, and the general kernel inlines
// every primitive (135 KB for fp32 Sum): the pair exchange ran 1.0-1.1 us faster per launch in a
// kernel holding only its own transfers (2 ranks, 128 B - 64 KiB, graph replay, same box:
// profiles/r04a_lat.txt).  kSetExchange: programs of `s`, `rrc` and the fused s + rrc only (the
// 2-rank pair exchange, xmlgen.allreduce_pair_oneshot; enqueue.cc picks it per launch).
enum : int { kSetAll = 0, kSetExchange = 1 };


// Error codes in DevComm::errWord
enum : uint32_t { kDevOk = 0, kDevTimeout = 1, kDevAbort = 2, kDevBadOp = 3 };

// Host-side kernel dispatch (kernels.hip)
typedef int (*LaunchFn)(const LaunchArgs& args, int gridBlocks, void* stream);
typedef int (*OneRankFn)(const void* src, void* dst, size_t n, uint64_t arg, int argIsPtr, void* stream);
OneRankFn getOneRankFn(int dtype);
constexpr int kQueryResidency = -1;  // LaunchFn(args, kQueryResidency, _) = resident workgroups per CU
LaunchFn getLaunchFn(int dtype, int redop, int proto);
LaunchFn getSmallLaunchFn(int dtype, int redop, int set);  // mscclSmallKernel (LL, Sum..Min, kSet*), or null
LaunchFn getFoldLaunchFn(int dtype, int redop);   // mscclFoldKernel (the flat tree), or null
// The pair kernel (mscclPairKernel): a launch whose every rank runs a pair-form schedule (every
// thread block: one fused s + rrc of one chunk at an affine chunk index, no dependency) in one
// pass: no program image, the first FIFO step's source loaded with the connection records.
LaunchFn getPairLaunchFn(int dtype, int redop);
// The two-phase fold (mscclTwoPhaseKernel, interpreter.h: runTwoPhase): a lowered schedule's
// large calls, LL, Sum..Min
LaunchFn getTwoPhaseLaunchFn(int dtype, int redop);
// The direct form of a Simple schedule (mscclDirectKernel, interpreter.h: DirectRunner), Sum..Min
LaunchFn getDirectLaunchFn(int dtype, int redop);
// the name of the first type whose kernel object was built with another RankWork layout, or null
const char* kernelLayoutMismatch();
// One-thread kernel that writes the GPU clock (s_memrealtime) to *hostWord (host-mapped):
// NPKit's host/GPU clock calibration.  Returns 0 on a successful launch.
int launchClockProbe(uint64_t* hostWord, void* stream);
// 16-B line atomicity probe (kernels_probe.hip, mscclAmdLineTearProbe)
int launchLineWriter(void* lines, int nLines, int iters, int blocks, void* stream);
int launchLineReader(const void* lines, int nLines, int iters, uint64_t ticks, unsigned long long* out, int blocks,
                     void* stream);

}  // namespace msccl

static_assert(sizeof(msccl::LaunchArgs) <= 4096, "kernel argument block must stay within 4 KiB");

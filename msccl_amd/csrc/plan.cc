#include "plan.h"

#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include <algorithm>
#include <string>

#include "debug.h"
#include "device/devcomm.h"

namespace msccl {

int refTypeSize(int t) {  // core.h:33-53
  switch (t) {
    case 0: case 1: return 1;
    case 6: case 9: return 2;
    case 2: case 3: case 7: return 4;
    case 4: case 5: case 8: return 8;
    default: return -1;
  }
}

bool inPlaceOf(int coll, const void* send, const void* recv, size_t count, int dtype, int rank) {
  const char* s = (const char*)send;
  const char* r = (const char*)recv;
  size_t ts = (size_t)refTypeSize(dtype);
  if (coll == kAllGather) return s == r + (size_t)rank * count * ts;
  if (coll == kReduceScatter) return r == s + (size_t)rank * count * ts;
  return s == r;
}

// parseList (tuning.cc:34-55): "^A,B" disables, "A,B" enables only those
static bool listEnables(const char* str, const char* name, bool def) {
  if (!str) return def;
  bool invert = str[0] == '^';
  std::string s(str + (invert ? 1 : 0));
  bool found = false;
  size_t p = 0;
  while (p <= s.size()) {
    size_t q = s.find(',', p);
    if (q == std::string::npos) q = s.size();
    if (!strcasecmp(s.substr(p, q - p).c_str(), name)) found = true;
    p = q + 1;
  }
  return invert ? !found : found;
}

static int getNthreads(const char* env) {  // NCCL_PARAM-style cached read; -2 = unset
  return (int)envInt(env, -2);
}

Knobs Knobs::fromEnv() {
  initEnv();  // ~/.nccl.conf, /etc/nccl.conf (the reference's initEnv, before any NCCL_PARAM read)
  Knobs k;
  memset(&k, 0, sizeof(k));
  // The reference runs an MSCCL AllReduce only when NCCL_ALGO lists MSCCL (algoEnable default 0,
  // tuning.cc:186; zeroed AllReduce bandwidths, tuning.cc:217), and never when a group holds more
  // than one op of the communicator (asyncOpCount > 1, enqueue.cc:448-460).  Here MSCCL is the
  // primary algorithm: on unless NCCL_ALGO excludes it, in any group.
  // MSCCL_AMD_REFERENCE_SELECTION=1 restores both reference rules.
  k.referenceSelection = envInt("MSCCL_AMD_REFERENCE_SELECTION", 0) != 0;
  k.mscclOn = listEnables(getenv("NCCL_ALGO"), "MSCCL", !k.referenceSelection);
  static const char* names[3] = {"LL", "LL128", "Simple"};
  for (int p = 0; p < 3; p++) k.protoOn[p] = listEnables(getenv("NCCL_PROTO"), names[p], true);
  k.nthreads = getNthreads("NCCL_NTHREADS");
  k.ll128Nthreads = getNthreads("NCCL_LL128_NTHREADS");
  k.buffSizes[kProtoLL] = envInt("NCCL_LL_BUFFSIZE", 8 * 512 * kFifoSteps * 16);
  k.buffSizes[kProtoLL128] = envInt("NCCL_LL128_BUFFSIZE", 120 * 640 * kFifoSteps * 8);
  k.buffSizes[kProtoSimple] = envInt("NCCL_BUFFSIZE", 1 << 22);
  k.simpleBuffEnv = getenv("NCCL_BUFFSIZE") != nullptr;
  k.ringChannels = (int32_t)envInt("MSCCL_AMD_RING_CHANNELS", 0);
  k.split = (int32_t)envInt("MSCCL_AMD_SPLIT", 0);
  k.targetWgs = (int32_t)envInt("MSCCL_AMD_TARGET_WGS", 0);  // 0: by protocol (chooseSplit)
  k.merge = (int32_t)envInt("MSCCL_AMD_MERGE", 0);
  k.ringFallback = envInt("MSCCL_AMD_RING_FALLBACK", 1) != 0;
  k.ll128Remote = envInt("MSCCL_AMD_LL128_REMOTE", 0) != 0;
  k.ringOn = listEnables(getenv("NCCL_ALGO"), "Ring", true);
  k.treeOn = listEnables(getenv("NCCL_ALGO"), "Tree", true);
  k.treeMaxBytes = envInt("MSCCL_AMD_TREE_MAX_BYTES", -1);  // -1: the defaults of makeRingPlan / makeFlatTreePlan
  k.smallKernel = envInt("MSCCL_AMD_SMALL_KERNEL", 1) != 0;
  k.pairKernel = envInt("MSCCL_AMD_PAIR_KERNEL", 1) != 0;
  k.fuse = envInt("MSCCL_AMD_FUSE", 1) != 0;
  k.treeFlat = envInt("MSCCL_AMD_TREE_FLAT", 1) != 0;
  k.lower = envInt("MSCCL_AMD_LOWER", 1) != 0;
  k.lowerMaxBytes = envInt("MSCCL_AMD_LOWER_MAX_BYTES", -1);  // -1: by rank count (lowerToFoldPlan)
  k.lowerLarge = envInt("MSCCL_AMD_LOWER_LARGE", 1) != 0;
  k.forceRemote = envInt("MSCCL_AMD_FORCE_REMOTE", 0) != 0;
  k.twoPhaseStep = (int32_t)envInt("MSCCL_AMD_TWO_PHASE_STEP", 0);
  k.direct = envInt("MSCCL_AMD_DIRECT", 1) != 0;
  return k;
}

bool useLocalSimpleFifo(bool oneGpu, const Knobs& k, const std::vector<Algorithm>& algos,
                        const std::vector<int>& sendRun) {
  if (!oneGpu || k.simpleBuffEnv) return false;
  for (size_t a = 0; a < algos.size(); a++)
    if (algos[a].proto == kProtoSimple && a < sendRun.size() && sendRun[a] > 2) return false;
  return true;
}

int chooseSplit(int maxBlocks, int coResident, const Knobs& kn, int proto, bool wide) {
  int k = 1;
  if (kn.split > 0) {
    while (k * 2 <= kMaxSplit && k * 2 <= kn.split) k *= 2;
    return k;
  }
  // Workgroups per GPU: one per CU for LL / LL128 schedules, two for Simple.  Same box, alternating
  // runs (profiles/r05g_target_wgs.txt): 8 co-resident ranks, LL fp16 all-pairs 2 MiB 48.0 ->
  // 41.8 us, 32 MiB 541 -> 532, RCCL's 8n-32tb file 602 -> 554 us (split 2 -> 1); the Simple C4
  // ring 1.49 ms at 512 against 1.76 at 256 (r05e_c4knobs.txt)
  const int64_t target = kn.targetWgs > 0 ? kn.targetWgs : proto == kProtoSimple || wide ? 512 : 256;
  int64_t per = (int64_t)std::max(1, maxBlocks) * std::max(1, coResident);
  while (k * 2 <= kMaxSplit && per * k * 2 <= target) k *= 2;
  return k;
}

static void argsCheck(const CallDesc& c, int64_t* count, int* dtype, int64_t* nBytes) {
  *nBytes = (int64_t)c.count * refTypeSize(c.dtype);
  *count = (int64_t)c.count;
  *dtype = c.dtype;
  if (c.coll == kAllGather || c.coll == kBroadcast || c.coll == kAllToAll) {
    *count = *nBytes;
    *dtype = 0;
  }
  if (c.coll == kAllGather || c.coll == kReduceScatter || c.coll == kAllToAll) *nBytes *= c.nRanks;
}

int selectAlgo(const std::vector<Algorithm>& algos, const std::vector<Registration>& regs, const CallDesc& c,
               const Knobs& k) {
  if (!(c.redop == 0 || c.redop == 1 || c.redop == 2 || c.redop == 3)) return -1;  // tuning.cc:345
  // NCCL_ALGO gates AllReduce only: "Only disable algo for Allreduce since others only have one"
  // (tuning.cc:216-217)
  if (!k.mscclOn && c.coll == kAllReduce) return -1;
  int64_t count, nBytes;
  int dt;
  argsCheck(c, &count, &dt, &nBytes);
  int64_t total = (c.coll == kAllToAll || c.coll == kAllGather || c.coll == kReduceScatter) ? count * c.nRanks : count;
  auto ok = [&](const Algorithm& a) {
    return a.valid && k.protoOn[a.proto] && a.coll == c.coll && a.inPlace == (int)c.inPlace &&
           a.ngpus == c.nRanks && a.nchunksPerLoop > 0 && total % a.nchunksPerLoop == 0;
  };
  if (c.customAlgo >= 0) {
    if (c.customAlgo < (int)algos.size() && algos[c.customAlgo].valid && algos[c.customAlgo].coll == kCustom) return c.customAlgo;
    return -1;
  }
  if (!regs.empty()) {  // MSCCL_CONFIG registrations (tuning.cc:350-363)
    for (auto& r : regs) {
      if (r.minBytes <= nBytes && (nBytes < r.maxBytes || r.maxBytes == -1)) {
        if (r.algoIndex < (int)algos.size() && ok(algos[r.algoIndex]) && k.protoOn[r.proto]) return r.algoIndex;
      }
    }
    return -1;
  }
  for (size_t i = 0; i < algos.size(); i++) {
    const Algorithm& a = algos[i];
    if (ok(a) && nBytes >= a.minBytes && nBytes < a.maxBytes) return (int)i;
  }
  return -1;
}

static int clampNthreads(int nt, int lo, int hi, int def) {  // tuning.cc:14-32
  if (nt > 0) {
    if (nt % kRefWarp != 0) return hi;
    if (nt > hi) return hi;
    if (nt < lo) return lo;
    return nt;
  }
  return def;
}

int makePlan(const std::vector<Algorithm>& algos, int algoIndex, int protoOverride, const CallDesc& c, const Knobs& k,
             Plan* p) {
  const Algorithm& a = algos[algoIndex];
  *p = Plan();
  p->algoIndex = algoIndex;
  p->proto = protoOverride >= 0 ? protoOverride : a.proto;
  argsCheck(c, &p->count, &p->dtype, &p->nBytes);
  int nt;
  if (p->proto == kProtoSimple) nt = clampNthreads(k.nthreads, 2 * kRefWarp, 512, 512);
  else if (p->proto == kProtoLL) nt = clampNthreads(k.nthreads, 2 * kRefWarp, 512, 512);
  else nt = clampNthreads(k.ll128Nthreads, 640 / 4, 640, 640);
  if (a.nThreads > 0) nt = std::min(nt, a.nThreads);
  if (p->proto == kProtoSimple) nt += kRefWarp;  // extra sync warp (enqueue.cc:516-517)
  p->refNthreads = nt;
  const int64_t* bs = k.buffSizes;
  int64_t stepSize = bs[p->proto] / kFifoSteps;
  int64_t chunkSteps = p->proto == kProtoSimple ? kChunkSteps : 1;
  int64_t chunkSize = stepSize * chunkSteps;
  int64_t chunkEff = chunkSize;
  if (p->proto == kProtoLL) chunkEff /= 2;
  if (p->proto == kProtoLL128) chunkEff = (chunkSize / 16) * 15;
  p->nchunksPerLoop = a.nchunksPerLoop;
  int ts = refTypeSize(p->dtype);
  if (p->nBytes % a.nchunksPerLoop != 0) {
    WARN("MSCCL: something went wrong. MSCCL algorithm needs the input buffer to be divisible by %d", a.nchunksPerLoop);
    return 3;
  }
  if (p->proto == kProtoSimple && chunkSize % ((nt - kRefWarp) * 8 / ts) != 0) {
    WARN("chunkSize (%ld) should be divisble by (nthreads-WARP_SIZE) (%d) for Simple protocol", (long)chunkSize, nt - kRefWarp);
    return 3;
  }
  int64_t mac = 0;
  if (p->nBytes > 0) {
    int64_t perChunk = (p->nBytes + a.nchunksPerLoop - 1) / a.nchunksPerLoop;
    mac = std::max<int64_t>(1, chunkEff / perChunk);
  }
  if (mac == 0) { WARN("MSCCL: something went wrong. Max allowed count is 0"); return 3; }
  if (mac >= kMaxCount) mac = kMaxCount - 1;
  p->maxAllowedCount = (int)mac;
  p->sizeMultiplier = (c.coll == kReduceScatter || c.coll == kAllGather || c.coll == kAllToAll) ? c.nRanks : 1;
  p->scratchNeeded = (size_t)p->nBytes * (size_t)a.nScratchChunks / (size_t)a.nchunksPerLoop;

  // interpreter parameters (msccl_interpreter.h:79-86)
  int64_t bytePerStep;
  if (p->proto == kProtoLL) {
    bytePerStep = bs[0] / kFifoSteps / 2;
    p->minChunk = (int64_t)nt * (8 / ts);
  } else if (p->proto == kProtoLL128) {
    bytePerStep = (bs[1] / kFifoSteps) * 15 / 16;
    p->minChunk = (int64_t)nt * ((8 * 15 * 8 / 16) / ts) / 2;
  } else {
    bytePerStep = bs[2] / kFifoSteps;
    p->minChunk = (int64_t)(nt - kRefWarp) * 8 / ts;
  }
  p->chunkSize = (int64_t)(int)(bytePerStep / ts * (p->proto == kProtoSimple ? kChunkSteps : 1));
  p->sizePerChunk = (p->count * p->sizeMultiplier) / a.nchunksPerLoop;
  p->nIters = p->chunkSize > 0 ? (int)((p->sizePerChunk + p->chunkSize - 1) / p->chunkSize) : 0;
  if (p->minChunk <= 0) p->minChunk = 1;
  return 0;
}

// The reference's tree AllReduce (all_reduce.h:103-298) on this build's chain (rank order, root
// 0; the reference's intra-node trees are chains too): chunk math of computeColl for the tree
// (enqueue.cc:634-644, Simple: the step halved while the loop is short relative to the tree
// depth, n here) and of runTreeUpDown/runTreeSplit (loopSize > size: chunkSize =
// divUp(size, nChannels * minChunkSize) * minChunkSize).
static int makeTreePlan(const CallDesc& c, const Knobs& k, Plan* p) {
  const int ts = refTypeSize(p->dtype);
  const int64_t C = p->ringChannels;
  int nt;
  int64_t chunk, minChunk;
  if (p->proto == kProtoLL) {
    nt = clampNthreads(k.nthreads, 2 * kRefWarp, 512, 512);
    chunk = k.buffSizes[kProtoLL] / kFifoSteps * 8 / 16 / ts;   // calcBytePerStep / sizeof(T)
    minChunk = (int64_t)nt * 8 / ts;                             // nthreads * calcBytePerGrain / sizeof(T)
  } else {
    nt = clampNthreads(k.nthreads, 2 * kRefWarp, 512, 512) + kRefWarp + 3 * kRefWarp;  // enqueue.cc:516-520
    int64_t cb = k.buffSizes[kProtoSimple] / kFifoSteps;         // stepSize, chunkSteps 1 for the tree
    const int64_t depth = c.nRanks;
    while (p->nBytes / (C * cb) < depth * 8 && cb > 131072) cb /= 2;
    while (p->nBytes / (C * cb) < depth * 4 && cb > 65536) cb /= 2;
    while (p->nBytes / (C * cb) < depth && cb > 32768) cb /= 2;
    chunk = cb / ts;                                             // lastChunkSize
    minChunk = (int64_t)(nt - 2 * kRefWarp) * 8 * (8 / ts);
  }
  if (C * chunk > p->count) chunk = (p->count + C * minChunk - 1) / (C * minChunk) * minChunk;
  p->refNthreads = nt;
  p->chunkSize = chunk;
  p->minChunk = minChunk;
  p->ringColl = kTreeAllReduce;
  return 0;
}

int makeFlatTreePlan(const CallDesc& c, const Knobs& k, Plan* p) {
  if (!k.treeFlat || p->proto != kProtoLL || c.nRanks < 2 || c.nRanks > kMaxReduceFusion || p->nBytes > (1ll << 30))
    return 1;
  int mode;
  if (p->ringColl == kTreeAllReduce) {
    if (c.redop > kDevMin) return 1;
    mode = kRingAllReduce;
  } else if (p->ringColl == kRingReduceScatter || p->ringColl == kRingAllGather) {
    if (p->ringColl == kRingReduceScatter && c.redop > kDevMin) return 1;  // pre / post ops: the ring
    // one hop instead of the ring's n - 1 over the whole LL range (profiles/r03_fold_xover.txt:
    // 8 ranks 64 KiB per rank 41.6 -> 17.6 us), or a rank's block up to MSCCL_AMD_TREE_MAX_BYTES
    if (k.treeMaxBytes >= 0 && p->nBytes / c.nRanks > k.treeMaxBytes) return 1;
    mode = p->ringColl;
  } else {
    return 1;
  }
  // It runs in its own kernel (interpreter.h: runFold) as one call over the whole buffer (at
  // most 1 GiB: 32-bit offsets); the fields below keep the MSCCL plan's form for introspection,
  // sizePerChunk = count being what the kernel reads.  Chunk math of makePlan for LL (enqueue.cc:591-734,
  // msccl_interpreter.h:79-86) with nchunksPerLoop 1 and the tree's thread count.
  const int ts = refTypeSize(p->dtype);
  const int nt = p->refNthreads;
  const int64_t stepSize = k.buffSizes[kProtoLL] / kFifoSteps;
  p->ringColl = kTreeFlat;
  p->flatColl = mode;
  p->ringChannels = 0;
  p->nchunksPerLoop = 1;
  p->sizeMultiplier = 1;
  p->maxAllowedCount = (int)std::min<int64_t>(kMaxCount - 1, std::max<int64_t>(1, (stepSize / 2) / std::max<int64_t>(1, p->nBytes)));
  p->chunkSize = (int64_t)(int)(stepSize / 2 / ts);
  p->minChunk = std::max<int64_t>(1, (int64_t)nt * (8 / ts));
  p->sizePerChunk = p->count;
  p->nIters = (int)((p->sizePerChunk + p->chunkSize - 1) / p->chunkSize);
  p->scratchNeeded = 0;
  return 0;
}

int64_t foldLinkCrossoverBytes(int nRanks) {
  if (nRanks <= 2) return -1;
  const double f = 2.0;  // LL: a 16-B line per 8-B payload
  const double bytesPerUs = kXgmiLinkOneWayGBs * 1e3;
  return (int64_t)((kInterpFixedUs + kXgmiHopUs) * bytesPerUs / (f * (1.0 - 2.0 / nRanks)));
}

int64_t defaultLowerMaxBytes(int nRanks, bool remote) {
  // Ranks on one GPU, where the fold beats the interpreted schedule (graph replay,
  // profiles/r04b_xover.txt, r04l_sweep.txt): 2 ranks up to a few KiB (the exchange-set kernel
  // runs the pair exchange itself in ~6.6 us from 8 KiB on), more ranks up to 128 KiB (16 fold
  // workgroups per rank, profiles/r04t_lat.txt: the one-shot 64 KiB 23.7 -> 11.3 us, the two-phase
  // all-pairs 128 KiB 17.9-21.1 -> 13.1; at 256 KiB 21.6 against 21.2, even)
  if (!remote || nRanks <= 2) return nRanks <= 2 ? (int64_t)(4 << 10) : (int64_t)(128 << 10);
  // Peers on other GPUs: the link model's crossover, rounded down to a power of two and capped at
  // the size where the fold kernel's 16 workgroups per rank stop keeping up on one GPU.  Two
  // ranks keep the co-resident value: the pair exchange is one hop with the fold's link bytes.
  const int64_t x = foldLinkCrossoverBytes(nRanks);
  int64_t p = 4 << 10;
  while (p * 2 <= x && p * 2 <= kFoldMaxBytesCap) p *= 2;
  return p;
}

int lowerToFoldPlan(const CallDesc& c, const Knobs& k, int classes, bool twoPhase, Plan* p) {
  const int64_t limit = k.lowerMaxBytes >= 0 ? k.lowerMaxBytes : defaultLowerMaxBytes(c.nRanks, c.remote);
  if (!k.lower || c.coll != kAllReduce || p->proto != kProtoLL || c.redop > kDevMin || p->nBytes > (1ll << 30))
    return 1;
  const int ts = refTypeSize(p->dtype);
  const int64_t pe = 16 / ts;
  if (p->nBytes > limit) {
    if (!k.lowerLarge) return 1;
    int mode;
    if (c.nRanks == 2) {
      mode = kLowerPair;  // any fold of two inputs: fn(x_0, x_1) == fn(x_1, x_0) (lower.cc)
    } else if (twoPhase && p->sizePerChunk % pe == 0 && p->nchunksPerLoop <= kMaxFoldChunks &&
               p->sizePerChunk / pe * (p->nchunksPerLoop / c.nRanks) <= (int64_t)INT32_MAX) {
      mode = kLowerTwoPhase;
    } else {
      return 1;
    }
    // one call over the whole buffer on the flat connections: no chunk loop, no FIFO merge rule,
    // no scratch; the fields keep makePlan's meaning for introspection
    p->lowerMode = mode;
    p->foldChunkPacks = mode == kLowerTwoPhase ? p->sizePerChunk / pe : 0;
    if (mode == kLowerPair) p->sizePerChunk = p->count;  // one chunk: the whole buffer
    p->ringColl = kTreeFlat;
    p->flatColl = kRingAllReduce;
    p->ringChannels = 0;
    p->maxAllowedCount = 1;
    p->scratchNeeded = 0;
    return 0;
  }
  if (classes > 1 && (p->sizePerChunk % pe != 0 || p->nchunksPerLoop > kMaxFoldChunks)) return 1;
  p->foldChunkPacks = classes > 1 ? p->sizePerChunk / pe : 0;
  // the fold kernel's chunk math (makeFlatTreePlan): one call over the whole buffer
  const int64_t stepSize = k.buffSizes[kProtoLL] / kFifoSteps;
  p->ringColl = kTreeFlat;
  p->flatColl = kRingAllReduce;
  p->ringChannels = 0;
  p->nchunksPerLoop = 1;
  p->sizeMultiplier = 1;
  p->maxAllowedCount = (int)std::min<int64_t>(kMaxCount - 1, std::max<int64_t>(1, (stepSize / 2) / std::max<int64_t>(1, p->nBytes)));
  p->chunkSize = (int64_t)(int)(stepSize / 2 / ts);
  p->minChunk = std::max<int64_t>(1, (int64_t)p->refNthreads * (8 / ts));
  p->sizePerChunk = p->count;
  p->nIters = (int)((p->sizePerChunk + p->chunkSize - 1) / p->chunkSize);
  p->scratchNeeded = 0;
  return 0;
}

int makeRingPlan(const CallDesc& c, const Knobs& k, Plan* p) {
  *p = Plan();
  p->algoIndex = -1;
  if (c.redop < 0 || c.redop > kDevSumPostDiv) return 5;
  if (c.redop == kDevSumPostDiv && !(c.dtype <= 5)) return 5;  // SumPostDiv is for integer types
  // Small AllReduces take the tree: every chain thread block runs one transfer per chunk where a
  // ring thread block runs 2(n-1), so the tree wins while latency dominates.  Measured on
  // co-resident ranks, fp16 (profiles/r02_fallback_ring_tree.txt): 2 ranks 128 B 11.7 -> 8.0 us,
  // 64 KiB ring ahead (16.3 vs 18.1); 8 ranks 128 B 35.9 -> 17.7 us, 64 KiB 52.6 -> 45.3 us,
  // 1 MiB ring ahead (64 vs 85).  Default threshold: 16 KiB per rank.  Calls the tree then runs
  // as the flat tree (makeFlatTreePlan: LL, Sum..Min, 2..16 ranks) take it over the whole LL
  // range (512 KiB): the one-hop fold kernel beats the LL ring there (fp16, co-resident,
  // profiles/r03_fold_xover.txt: 2 ranks 256 KiB 60.0 -> 25.3 us, 8 ranks 64 KiB 60.8 -> 16.4,
  // 16 ranks 256 KiB 129 -> 108).
  if (c.coll == kAllReduce) p->ringColl = kRingAllReduce;
  else if (c.coll == kReduceScatter) p->ringColl = kRingReduceScatter;
  else if (c.coll == kAllGather) p->ringColl = kRingAllGather;
  else return 5;
  argsCheck(c, &p->count, &p->dtype, &p->nBytes);   // AllGather: bytes, int8 (argcheck.cc:44-51)
  const int ts = refTypeSize(p->dtype);
  const bool llOk = k.protoOn[kProtoLL], simpleOk = k.protoOn[kProtoSimple];
  if (!llOk && !simpleOk) return 5;
  p->proto = (llOk && (p->nBytes <= (512 << 10) || !simpleOk)) ? kProtoLL : kProtoSimple;
  const bool flatTree = k.treeFlat && p->proto == kProtoLL && c.redop <= kDevMin && c.nRanks >= 2 &&
                        c.nRanks <= kMaxReduceFusion;
  const int64_t treeMax = k.treeMaxBytes >= 0 ? k.treeMaxBytes
                          : flatTree          ? (int64_t)(512 << 10)
                                              : (int64_t)16384 * c.nRanks;
  const bool tree = c.coll == kAllReduce && k.treeOn &&
                    (!k.ringOn || (int64_t)c.count * refTypeSize(c.dtype) <= treeMax);
  if (!tree && !k.ringOn) return 5;
  const int64_t forced = k.ringChannels;
  int64_t ch = forced > 0 ? forced : std::max<int64_t>(1, p->nBytes >> 18);
  p->ringChannels = (int)std::max<int64_t>(1, std::min<int64_t>(kRingChannels, ch));
  if (tree) return makeTreePlan(c, k, p);
  const int64_t* bs = k.buffSizes;
  int nt;
  if (p->proto == kProtoLL) {
    nt = clampNthreads(k.nthreads, 2 * kRefWarp, 512, 512);
    p->chunkSize = bs[0] / kFifoSteps / 2 / ts;             // calcBytePerStep (primitives.h:49-51)
    p->minChunk = (int64_t)nt * 8 / ts;                      // all_reduce.h:30-31
  } else {
    nt = clampNthreads(k.nthreads, 2 * kRefWarp, 512, 512) + kRefWarp;  // enqueue.cc:516-517
    p->chunkSize = bs[2] / kFifoSteps / ts * kChunkSteps;   // x ALLREDUCE/REDUCESCATTER/ALLGATHER_CHUNKSTEPS
    p->minChunk = (int64_t)(nt - kRefWarp) * 8 / ts;         // all_reduce.h:45 rounding unit
  }
  p->refNthreads = nt;
  p->maxAllowedCount = 1;
  p->sizeMultiplier = 1;
  if (p->proto == kProtoLL && p->ringColl != kRingAllReduce) {
    // enqueue.cc:653-658 with nchunksPerLoop = nRanks (ring pattern)
    const int64_t stepSize = bs[0] / kFifoSteps;
    const int64_t sliceSize = stepSize * 8 / 16;
    const int64_t loop = (int64_t)p->ringChannels * c.nRanks * sliceSize;
    int64_t last = (p->nBytes - (p->nBytes / loop) * loop + (int64_t)p->ringChannels * c.nRanks - 1) /
                   ((int64_t)p->ringChannels * c.nRanks);
    const int64_t align = (int64_t)nt * 8;
    last = (last + align - 1) / align * align;
    p->ringLastChunk = last / ts;
  }
  return 0;
}

// The direct form (lower.h: DirectLowering) for this call of a Simple schedule: op Sum..Min, every
// interpreter iteration moving at least nthreads elements per chunk (there Simple's `re` folds
// (s_0 (+) ...) (+) d, the order the analysis read; below it the reference takes the per-element
// d-first path, msccl_interpreter.h:157-170), and with several fold orders output chunks of whole
// 16-B packs (each pack folds in its chunk's order).  Sets p->directOk; the launch decides
// (enqueue.cc: launchGroup: every rank of the communicator in it).
static void directEligible(const CallDesc& c, const Knobs& k, int classes, Plan* p) {
  p->directOk = false;
  if (!k.direct || p->proto != kProtoSimple || c.redop > kDevMin || p->nBytes > (1ll << 30)) return;
  const int64_t sp = p->sizePerChunk, cs = p->chunkSize;
  if (c.coll != kAllGather) {
    if (sp < p->refNthreads) return;
    const int64_t tail = cs > 0 ? sp % cs : 0;
    if (tail != 0 && tail < p->refNthreads) return;
  }
  const int64_t pe = 16 / refTypeSize(p->dtype);
  if (classes > 1 && (sp % pe != 0 || sp / pe > INT32_MAX)) return;
  p->directChunkPacks = classes > 1 ? sp / pe : 0;
  p->directOk = true;
}

int planCall(const PlanContext& ctx, const CallDesc& c, bool asyncMany, Plan* p) {
  const std::vector<Algorithm>& algos = *ctx.algos;
  const Knobs& k = *ctx.knobs;
  // the ring / tree fallback, or its flat form (one hop) when the flat group exists
  auto fallback = [&]() {
    if (!ctx.ringFallback || makeRingPlan(c, k, p) != 0) return false;
    if (ctx.flat) makeFlatTreePlan(c, k, p);
    return true;
  };
  if (asyncMany && k.referenceSelection && c.customAlgo >= 0) {
    WARN("MSCCL algorithms is not supposed to be used in async mode!");  // enqueue.cc:448-451
    return 5;  // ncclInvalidUsage
  }
  const int idx = asyncMany && k.referenceSelection ? -1 : selectAlgo(algos, *ctx.regs, c, k);
  if (idx < 0) {
    // no MSCCL algorithm matches: the reference falls back to its ring (enqueue.cc:461-476)
    if (fallback()) {
      // the ring's Simple ReduceScatter / AllGather on ranks that share one launch: the direct form
      // (its values are the ring's: a block's fold along the ring from the rank after its owner,
      // reduce_scatter.h:50-65; the AllGather's copies), decided at the launch (enqueue.cc)
      if (ctx.ringDirect && k.direct && p->proto == kProtoSimple && c.redop <= kDevMin && p->nBytes <= (1ll << 30) &&
          (p->ringColl == kRingReduceScatter || p->ringColl == kRingAllGather)) {
        p->directOk = true;
        p->directChunkPacks = 0;
      }
      INFO(kSubColl, "MSCCL: no algorithm matches coll=%d count=%zu type=%d; %s fallback (%s, %d channels)", c.coll,
           c.count, c.dtype, p->ringColl == kTreeFlat ? "flat" : p->ringColl == kTreeAllReduce ? "tree" : "ring",
           p->proto == kProtoLL ? "LL" : "Simple", p->ringChannels);
      return 0;
    }
    WARN("MSCCL: no loaded algorithm matches coll=%d count=%zu type=%d op=%d inplace=%d nranks=%d "
         "and the ring fallback %s", c.coll, c.count, c.dtype, c.redop, (int)c.inPlace, c.nRanks,
         ctx.ringFallback ? "does not support it" : "is disabled (MSCCL_AMD_RING_FALLBACK=0)");
    return 5;
  }
  int protoOverride = -1;
  for (auto& r : *ctx.regs)
    if (r.algoIndex == idx) protoOverride = r.proto;
  if ((protoOverride >= 0 ? protoOverride : algos[idx].proto) == kProtoLL128 && c.remote && !k.ll128Remote) {
    // The CDNA4 LL128 line relies on a 16-B store arriving untorn.  That is observed for local
    // HBM, not shown for xGMI peer stores; the reference likewise enables LL128 only where its
    // line atomicity holds (tuning.cc:210-214).  Run the schedule with LL (same values for the
    // commutative ops MSCCL admits) unless MSCCL_AMD_LL128_REMOTE=1.
    static bool warned = false;
    if (!warned) {
      warned = true;
      WARN("MSCCL: algorithm %s is LL128 and peers are on other GPUs; running it with LL "
           "(MSCCL_AMD_LL128_REMOTE=1 keeps LL128)", algos[idx].name.c_str());
    }
    protoOverride = kProtoLL;
  }
  const int r = makePlan(algos, idx, protoOverride, c, k, p);
  if (r != 0) return r;
  const int dcls = ctx.directClasses && (size_t)idx < ctx.directClasses->size() ? (*ctx.directClasses)[idx] : 0;
  if (dcls > 0 && ctx.oneLaunch) directEligible(c, k, dcls, p);
  const int classes = ctx.foldClasses && (size_t)idx < ctx.foldClasses->size() ? (*ctx.foldClasses)[idx] : 0;
  const bool twoPhase = ctx.foldTwoPhase && (size_t)idx < ctx.foldTwoPhase->size() && (*ctx.foldTwoPhase)[idx];
  if (classes > 0 && ctx.flat && lowerToFoldPlan(c, k, classes, twoPhase, p) == 0) {
    // a one-hop schedule (lower.cc): the fold kernel computes its values in one hop; larger calls
    // the pair or the two-phase kernel
    INFO(kSubColl, "MSCCL: %s count=%zu runs lowered (%s)", algos[idx].name.c_str(), c.count,
         p->lowerMode == kLowerPair ? "pair exchange" : p->lowerMode == kLowerTwoPhase ? "two-phase fold" : "one-hop fold");
    return 0;
  }
  if (p->scratchNeeded > ctx.scratchSize) {
    // The scratch is sized from the XMLs' maxBytes at init (init.cc:809-835), so this only
    // happens when MSCCL_AMD_MAX_SCRATCH capped it.  The reference reports ncclInternalError
    // (enqueue.cc:580-589); the capped schedule is treated as not matching instead.
    const size_t need = p->scratchNeeded;
    if (fallback()) {
      INFO(kSubColl, "MSCCL: scratch %zu < %zu needed (MSCCL_AMD_MAX_SCRATCH); ring fallback", ctx.scratchSize, need);
      return 0;
    }
    WARN("MSCCL: MSCCL scratch pad size is smaller than expected %zu < %zu", ctx.scratchSize, need);
    return 3;  // ncclInternalError
  }
  return 0;
}

}  // namespace msccl

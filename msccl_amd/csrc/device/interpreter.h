// MSCCL schedule interpreter for gfx950.
//
// Behaviour follows the reference interpreter collectives/device/msccl_interpreter.h:66-205:
//   * outer loop over gridOffset in steps of chunkSize; per-protocol realChunkSize/nelem
//     (msccl_interpreter.h:105-113);
//   * per transfer: wait on dependency flags COMPUTE_FLAG(workIndex, iter, step) of other
//     thread blocks of the same rank (123-140), split `count` by mscclMaxAllowedCount (146-150),
//     dispatch to the primitive, publish the own flag when hasdep (198-201);
//   * reductions: LL order acc=d, acc=fn(acc,s_i) (prims_ll.h:347-362), LL128 acc=fn(s_i,acc)
//     (prims_ll128.h:381-392), Simple order (s0(+)s1..)(+)d (prims_simple.h:258-263),
//     per-element d-first path o=fn(s_i,o) when thisNelem < nthreads (157-170);
//   * recv-reduce: LL fn(peer, local) (prims_ll.h:282-287), Simple fn(local, peer).
//
// MI355X-native execution: wave64 workgroups of kNT threads, 16-B packs per lane, buffer
// loads/stores with explicit cache-policy bits, LL lines polled two at a time with a single
// wait, FIFO flow control through head/tail words in uncached memory, bounded spins.
//
// Work split.  One XML thread block may run as `split` workgroups.  Workgroup k owns, inside
// every MSCCL chunk, the k-th contiguous 1/split of that chunk's 16-B packs ("position within
// the chunk").  Every data movement of an MSCCL schedule preserves an element's position
// inside its chunk (a transfer moves whole chunks, offsets are chunk-granular), so workgroup k
// only ever reads what workgroup k of the same or another thread block (or rank) wrote: each
// workgroup has its own sub-connection (FIFO, head/tail, step counter) and its own dependency
// flag, and no transfer ever needs another workgroup's data.  A launch uses split = 1 whenever
// a chunk is not a whole number of packs.
#pragma once
#include "msccl_amd_npkit.h"
#include "primitives.h"

namespace msccl {

enum : int { tSend = 0, tRecv = 1, tRCS = 2, tRRS = 3, tRRC = 4, tRRCS = 5, tCpy = 6, tRe = 7, tCopySend = 9,
             tSendRrc = 10 /* s fused with the rrc after it (transport.cc: fusableTbs) */,
             tSendCpy = 11 /* s fused with the cpy of the same source after it: a copy-send */ };
enum : int { pLL = 0, pLL128 = 1, pSimple = 2 };

struct alignas(16) BlockShared {
  u32x4 img[kMaxImage16];  // this workgroup's thread-block image (devcomm.h: DevTbHeader)
  DevSendConn sconn;       // its connection records, copied once per launch (no global load of
  DevRecvConn rconn;       // connection metadata on the primitives' critical path)
  uint64_t seen[2];        // send head / recv tail last observed
  uint64_t epoch;
  uint32_t aborted;
  // MSCCL_AMD_TRACE=1: 10-ns ticks the polling lane spent waiting in this primitive call for the
  // Simple tail (data) and for send credit (head), saturating; in the padding of the struct
  uint16_t waitTail, waitHead;
};

// The flat tree's fold kernel (Interp::runFold), besides BlockShared: per peer, its send and recv
// connection records and this step's FIFO slots.
struct alignas(16) FoldShared {
  DevSendConn foldSend[kMaxFoldPeers];
  DevRecvConn foldRecv[kMaxFoldPeers];
  struct Peer {
    LLLine* out;        // send slot of this step (peer memory)
    const LLLine* in;   // recv slot of this step
    uint32_t sflag, rflag;
  } fold[kMaxFoldPeers];
  Peer fold2[kMaxFoldPeers];  // the two-phase fold: the second slot of the step (the owners' results)
  uint8_t perm[kMaxFoldPeers + 1];  // peer record of each fold position (the own input skipped)
  // a lowered schedule folding its chunks in several orders (lower.cc: classes): per class the
  // peer record of each fold position and the position of the own input; the class of each chunk
  uint8_t cperm[kMaxFoldClasses][kMaxFoldPeers + 1];
  uint8_t cown[kMaxFoldClasses];
  uint8_t chunkClass[kMaxFoldChunks];
};

__device__ __forceinline__ uint64_t computeFlag(uint64_t workIndex, uint64_t iter, uint64_t step) {
  return workIndex * (65536ull * 256ull) + iter * 256ull + step;  // msccl_interpreter.h:14-16
}

// LL line index of (pack p, half h): each group of 64 packs stores its first lines in 64
// consecutive lines and its second lines in the next 64, so a wave's stores/loads of one half
// are a contiguous 1 KiB.
__device__ __forceinline__ int llLineIdx(int p, int h) { return ((p >> 6) << 7) + (h << 6) + (p & 63); }

// a / b for a >= 0, b > 0: a shift when b is a power of two (the usual case for chunk and split
// sizes), so the iteration prologue does not pay for 64-bit software divisions
__device__ __forceinline__ int64_t divNonNeg(int64_t a, int64_t b) {
  if ((b & (b - 1)) == 0) return a >> (63 - __builtin_clzll((uint64_t)b));
  return a / b;
}

// The packs of one primitive call that this workgroup owns: `count` chunks of Q packs each,
// positions [q0, q0 + Lq) of every chunk.  Sub-local pack s maps to op pack bufPack(s).
struct Shape {
  int n;      // elements of the whole call (bound for tails)
  int Q;      // packs per chunk
  int q0, Lq; // owned positions
  int npk;    // owned packs = count * Lq
  __device__ __forceinline__ int bufPack(int s) const {
    if (Lq == Q) return s;  // split == 1 or a whole chunk: contiguous
    int c = s / Lq;
    return c * Q + q0 + (s - c * Lq);
  }
};

template <typename T, int OP, int PROTO>
struct Interp {
  using F = Fn<T, OP>;
  using PP = PrePost<T, OP>;
  static constexpr int TS = sizeof(T);
  static constexpr int PE = 16 / TS;  // elements per 16-B pack
  static constexpr int U = 4;         // packs per lane per pass (memory-level parallelism)
#ifndef MSCCL_SIMPLE_COPY_U
#define MSCCL_SIMPLE_COPY_U 4
#endif
  static constexpr int kSimpleCopyU = MSCCL_SIMPLE_COPY_U;  // Simple copies (simpleOp): packs per lane per pass

  BlockShared* sh;
  DevComm* comm;
  DevSendConn* sc;   // LDS copies (read-only in the primitives)
  DevRecvConn* rc;
  const DevTransfer* tr;  // the program in LDS (BlockShared::img)
  const int16_t* depBid;
  const int16_t* depStep;
  const int16_t* red;
  DevSendConn* scG;  // global connection state (step counters written back at the end)
  DevRecvConn* rcG;
  uint64_t sendStep, recvStep;
  uint64_t headSeen, tailSeen;  // credit / Simple data known available without polling
  uint64_t t0;
  uint64_t timeoutTicks;  // 0 = wait for ever (DevComm::timeoutTicks)
  uint32_t llFlagMask;    // LL / LL128 flag = (step + 1) & llFlagMask (NCCL_LL_FLAG, devcomm.h:56-63)
  uint32_t llCleanMask;   // cleanup steps: (step & mask) == mask (NCCL_LL_CLEAN_MASK)
  uint64_t redArg;        // PreMulSum scale bits / SumPostDiv rank count (RankWork::redOpArg)
  int tid;
  int refNthreads;
  TraceEvent* trace;  // this workgroup's trace slot (null = tracing off)
  int nev, maxEv;
  NpkitEvent* nkBuf;  // NPKit buffer of this thread block (null: off, or not the tb's sub 0)
  uint64_t* nkHeadG;  // its persistent event count
  uint64_t nkHead;
  int nkCap;

  // NPKit event (the reference's NpKit::CollectGpuEvent, npkit.h:26-37): thread 0 writes, every
  // thread keeps the count so it stays uniform
  __device__ __forceinline__ void nk(uint8_t type, uint64_t size, uint64_t ts) {
    if (nkBuf != nullptr) {
      if (tid == 0 && nkHead < (uint64_t)nkCap) {
        NpkitEvent e;
        e.bits = (uint64_t)type | ((size > 0xFFFFFFFFull ? 0xFFFFFFFFull : size) << 8);
        e.ts = ts;
        nkBuf[nkHead] = e;
      }
      nkHead++;
    }
  }
  __device__ __forceinline__ void nk(uint8_t type, uint64_t size) {
    if (nkBuf != nullptr) nk(type, size, __builtin_amdgcn_s_memrealtime());
  }
  // <primitive>_ENTRY of a transfer type (prims_ll.h:455-536; _EXIT = _ENTRY + 1)
  static __device__ __forceinline__ uint8_t nkPrim(int type) {
    switch (type) {
      case tSend: return NPKIT_EVENT_SEND_ENTRY;
      case tRecv: return NPKIT_EVENT_RECV_ENTRY;
      case tRCS: return NPKIT_EVENT_RECV_COPY_SEND_ENTRY;
      case tRRS: return NPKIT_EVENT_RECV_REDUCE_SEND_ENTRY;
      case tRRC:
      case tSendRrc: return NPKIT_EVENT_RECV_REDUCE_COPY_ENTRY;
      case tRRCS: return NPKIT_EVENT_RECV_REDUCE_COPY_SEND_ENTRY;
      case tCpy: return NPKIT_EVENT_LOCAL_COPY_ENTRY;
      case tCopySend:
      case tSendCpy: return NPKIT_EVENT_COPY_SEND_ENTRY;
      default: return NPKIT_EVENT_REDUCE_ENTRY;
    }
  }

  // MSCCL_LAT_TRACE (a measurement build, tools/lat_trace.py): timestamps at fixed points of a
  // small call.  Each point is a global store, whose completion later vmcnt(0) waits include, so
  // the points shift the times they measure by up to a store's round trip.
#ifdef MSCCL_LAT_TRACE
#define LAT_EV(T) ev((T), 0, 0)
#else
#define LAT_EV(T) ((void)0)
#endif
  __device__ __forceinline__ void ev(uint16_t type, uint16_t step, uint32_t arg) {
    if (trace != nullptr && tid == 0 && nev < maxEv) {
      TraceEvent e;
      e.ts = __builtin_amdgcn_s_memrealtime();
      e.type = type;
      e.step = step;
      e.arg = arg;
      trace[nev++] = e;
    }
  }

  // ---------------------------------------------------------------- spins / abort
  // Every poll loop owns a Spin.  Each 1024 polls check the host-mapped abort word
  // (ncclCommAbort) and, when MSCCL_AMD_TIMEOUT_SEC > 0, how long THIS wait has lasted (the
  // clock starts at the wait's first check, not at the launch).  The default, 0, waits for ever
  // as the reference does (prims_*.h checkAbort only polls the abort flag).  On abort or timeout
  // the error is recorded for ncclCommGetAsyncError and every later wait of the workgroup gives
  // up at once; the host then refuses further collectives on the communicator (enqueue.cc).
  struct Spin {
    uint32_t n = 0;
    uint64_t start = 0;
  };
  __device__ __forceinline__ bool spinAbort(Spin& sp) {
    if ((++sp.n & 1023u) != 0) return false;
    if (sh->aborted) return true;
    uint32_t code = kDevOk;
    if (atomicLoadSys32(comm->abortFlag)) {
      code = kDevAbort;
    } else if (timeoutTicks != 0) {
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (sp.n == 1024u) sp.start = now;
      else if (now - sp.start > timeoutTicks) code = kDevTimeout;
    }
    if (code != kDevOk) {
      sh->aborted = 1;
      atomicStoreSys32(comm->errWord, code);
      return true;
    }
    __builtin_amdgcn_s_sleep(1);
    return false;
  }

  static __device__ __forceinline__ uint16_t addTicks(uint16_t acc, uint64_t since) {
    const uint64_t d = acc + (__builtin_amdgcn_s_memrealtime() - since);
    return (uint16_t)(d > 0xFFFF ? 0xFFFF : d);
  }

  // Send credit: the receiver has freed slot `sendStep` once head + SLOTS > sendStep.  The
  // last head seen is kept (and persisted in the connection), so most steps need no poll of the
  // remote word, whose round trip is the largest part of a small message's latency.
  template <int SLOTS>
  __device__ __forceinline__ void waitSendCredit() {
    if (headSeen + SLOTS >= sendStep + 1) return;
    if (tid == 0) {
      Spin spins;
      uint64_t h;
      const uint64_t tw = trace != nullptr ? __builtin_amdgcn_s_memrealtime() : 0;
      while ((h = atomicLoadSys(sc->head)) + SLOTS < sendStep + 1) {
        if (spinAbort(spins)) break;
      }
      if (trace != nullptr) sh->waitHead = addTicks(sh->waitHead, tw);
      sh->seen[0] = h;
    }
    __syncthreads();
    headSeen = uni(sh->seen[0]);
  }
  // Simple data: the sender has posted step recvStep once tail > recvStep.  Hand-off forms
  // ("Simple hand-off"):
  //   producer on this GPU (remote == 0): the MI355X guide's sc0 sc1 form, table row 1 -- every
  //     FIFO store is an sc0 sc1 16-B store to uncached memory, drained by every storing wave,
  //     then a workgroup barrier and ONE lane's sc0 sc1 tail store; here ONE lane polls the tail
  //     with sc0 sc1 loads and the other waves load the slot (sc0 sc1) after the barrier it then
  //     joins.  No fence on either side.
  //   producer on another GPU (remote == 1): the sender's system-scope release before the tail
  //     (prims_simple.h:218) pairs with a system-scope acquire here, issued by the polling lane
  //     before the barrier.
  //   remote == 2 (MSCCL_AMD_SIMPLE_FENCE=1, measurement only): agent-scope fences on a local
  //     connection.
  // A step already covered by an earlier tail value was handed off with that value.
  __device__ __forceinline__ void waitRecvTail() {
    if (tailSeen >= recvStep + 1) return;
    if (tid == 0) {
      Spin spins;
      uint64_t t;
      const uint64_t tw = trace != nullptr ? __builtin_amdgcn_s_memrealtime() : 0;
      while ((t = atomicLoadSys(rc->tail)) < recvStep + 1) {
        if (spinAbort(spins)) break;
      }
      if (trace != nullptr) sh->waitTail = addTicks(sh->waitTail, tw);
      if (rc->remote == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      else if (rc->remote == 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      sh->seen[1] = t;
    }
    __syncthreads();
    tailSeen = uni(sh->seen[1]);
  }

  // ---------------------------------------------------------------- pack helpers
  __device__ __forceinline__ u32x4 loadPartial(__amdgpu_buffer_rsrc_t r, int e0, int ne) {
    T v[PE];
#pragma unroll
    for (int i = 0; i < PE; i++) {
      if (i < ne) v[i] = ldElem<T>(r, (uint32_t)(e0 + i) * TS);
      else __builtin_memset(&v[i], 0, TS);
    }
    u32x4 o;
    __builtin_memcpy(&o, v, 16);
    return o;
  }
  __device__ __forceinline__ void storePartial(__amdgpu_buffer_rsrc_t r, int e0, int ne, u32x4 x) {
    T v[PE];
    __builtin_memcpy(v, &x, 16);
#pragma unroll
    for (int i = 0; i < PE; i++)
      if (i < ne) stElem<T>(r, (uint32_t)(e0 + i) * TS, v[i]);
  }
  // op pack B of a buffer holding n elements
  __device__ __forceinline__ u32x4 loadPack(__amdgpu_buffer_rsrc_t r, bool vec, int B, int n) {
    int e0 = B * PE;
    int ne = n - e0;
    if (vec && ne >= PE) return ld16<kAuxLocal>(r, (uint32_t)e0 * TS);
    return loadPartial(r, e0, ne < PE ? ne : PE);
  }
  __device__ __forceinline__ void storePack(__amdgpu_buffer_rsrc_t r, bool vec, int B, int n, u32x4 x) {
    int e0 = B * PE;
    int ne = n - e0;
    if (vec && ne >= PE) st16<kAuxLocal>(r, (uint32_t)e0 * TS, x);
    else storePartial(r, e0, ne < PE ? ne : PE, x);
  }
  static __device__ __forceinline__ bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

  // ---------------------------------------------------------------- LL / LL128 protocols
  // One primitive call is cut into FIFO steps of at most one slot (slotPacks packs); sender and
  // receiver own the same packs, so they agree on the number of steps.  Two line formats share
  // the LL FIFO memory:
  //   LL    (prims_ll.h):  a 16-B line = two 8-B {4-B data, 4-B flag} granules; pack p of a step
  //                        occupies lines llLineIdx(p, 0/1).
  //   LL128 (CDNA4 form):  a 16-B line = {12 B data, 4-B flag}; 3 packs (12 dwords) travel as a
  //                        unit of 4 lines.  The reference's LL128 (prims_ll128.h) relies on NVLink
  //                        delivering a warp's 128-B line whole; CDNA4 documents no such
  //                        guarantee, and a 16-B aligned store is the unit observed untorn on
  //                        gfx950.  So the flag guards 12 B instead of 120 B: payload 75 % of the
  //                        wire bytes instead of LL's 50 %.
  // The values are the protocol's: recv-reduce fn(peer, local) for both.
  static constexpr bool kL16 = PROTO == pLL128;

  // LL128 line of (unit u, line j): 64 units keep line j of each in one contiguous 1 KiB
  static __device__ __forceinline__ int l16LineIdx(int u, int j) { return ((u >> 6) << 8) + (j << 6) + (u & 63); }
  static __device__ __forceinline__ int l16Lines(int nv) { return nv == 3 ? 4 : nv + 1; }  // lines for nv packs

  // FUSED (tSendRrc, RECV = SEND = SRC = DST = 1): send the source, receive the peer's same step,
  // dst = fn(peer, source): the s and rrc of one exchange in one pass over the source.
  template <int RECV, int SEND, int SRC, int DST, int FUSED = 0>
  __device__ void llOp(const T* src, T* dst, const Shape s) {
    constexpr int E = 8 / TS;  // elements per LL line
    const int nlinesFull = (s.n + E - 1) / E;
    const int slotLines = uni(SEND ? sc->llSlotLines : rc->llSlotLines);
    const int slotPacks = kL16 ? (slotLines / 256) * 64 * 3 : slotLines / 2;
    __amdgpu_buffer_rsrc_t srs, drs, frs;
    if (SRC) srs = makeRsrc(src);
    if (DST) drs = makeRsrc(dst);
    const bool vec = (!SRC || aligned16(src)) && (!DST || aligned16(dst));
    int s0 = 0;
    do {
      const int s1 = s.npk - s0 < slotPacks ? s.npk : s0 + slotPacks;
      if (SEND) waitSendCredit<kLLFifoSlots>();
      LLLine* rslot = nullptr;
      uint32_t rflag = 0, sflag = 0;
      if (RECV) {
        rslot = rc->ll + (recvStep % kLLFifoSlots) * (uint64_t)rc->llSlotLines;
        rflag = (uint32_t)(recvStep + 1) & llFlagMask;
      }
      if (SEND) {
        frs = makeRsrc(sc->ll + (sendStep % kLLFifoSlots) * (uint64_t)sc->llSlotLines);
        sflag = (uint32_t)(sendStep + 1) & llFlagMask;
      }
      if constexpr (kL16) {
        l16Step<RECV, SEND, SRC, DST>(srs, drs, frs, rslot, rflag, sflag, vec, s, s0, s1);
      } else {
        llStep<RECV, SEND, SRC, DST, FUSED>(srs, drs, frs, rslot, rflag, sflag, vec, s, s0, s1, nlinesFull);
      }
      if (SEND) {
        if ((sendStep & llCleanMask) == llCleanMask) {
          // LL cleanup (prims_ll.h:90-97): stamp every unused line of the slot with this flag
          const int units = (s1 - s0 + 2) / 3;
          for (int l = tid; l < slotLines; l += kNT) {
            bool used;
            if constexpr (kL16) {
              const int u = ((l >> 8) << 6) + (l & 63), j = (l >> 6) & 3;
              used = u < units && j < l16Lines(min(3, s1 - s0 - 3 * u));
            } else {
              const int q = ((l >> 7) << 6) + (l & 63), h = (l >> 6) & 1;
              used = s0 + q < s1 && 2 * s.bufPack(s0 + q) + h < nlinesFull;
            }
            if (!used) st16<kAuxFifo>(frs, (uint32_t)l * 16, (u32x4){0, sflag, 0, sflag});
          }
        }
        sendStep++;
      }
      if (RECV) {
        recvStep++;
        __syncthreads();
        if (tid == 0) atomicStoreSys(rc->remoteHead, recvStep);
      }
      s0 = s1;
    } while (s0 < s.npk);
  }

  // ---------------------------------------------------------------- fused exchange (tSendRrc, LL)
  // The s and rrc of one exchange (transport.cc: fusableTbs), the send one FIFO step ahead of the
  // receive.  Iteration k issues together the source loads of send step k + 1 and the line polls
  // of receive step k, then stores fn(peer, source) of step k, whose source is still in
  // registers from iteration k - 1, and the lines of step k + 1.  One memory round trip per step
  // and the source is read once: 6 S HBM bytes per rank for the pair exchange instead of 7 S.
  // Steps are cut as llOp cuts the s and the rrc (one pass per step: slotPacks <= kNT * U), so
  // the peer may run either form.
  // packs of FIFO step j of a call: B = op pack, act = in this step, two = second line used
  __device__ __forceinline__ void llStepPacks(const Shape& s, int slotPacks, int nlinesFull, int j, int (&B)[U],
                                              bool (&act)[U], bool (&two)[U]) {
    const int s0 = j * slotPacks, n = min(s.npk - s0, slotPacks);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int q = tid + u * kNT;
      act[u] = q < n;
      B[u] = act[u] ? s.bufPack(s0 + q) : 0;
      two[u] = act[u] && 2 * B[u] + 1 < nlinesFull;
    }
  }
  // lines of one send step (pack q of the step -> llLineIdx(q, h)), then LL cleanup and the step
  __device__ __forceinline__ void llSendLines(const Shape& s, int slotLines, int nlinesFull, int s0, int s1,
                                              const bool (&act)[U], const bool (&two)[U], const u32x4 (&v)[U]) {
    const __amdgpu_buffer_rsrc_t frs = makeRsrc(sc->ll + (sendStep % kLLFifoSlots) * (uint64_t)slotLines);
    const uint32_t sflag = (uint32_t)(sendStep + 1) & llFlagMask;
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (!act[u]) continue;
      const int q = tid + u * kNT;
      st16<kAuxFifo>(frs, (uint32_t)llLineIdx(q, 0) * 16, (u32x4){v[u].x, sflag, v[u].y, sflag});
      if (two[u]) st16<kAuxFifo>(frs, (uint32_t)llLineIdx(q, 1) * 16, (u32x4){v[u].z, sflag, v[u].w, sflag});
    }
    if ((sendStep & llCleanMask) == llCleanMask) {  // prims_ll.h:90-97, as in llOp
      for (int l = tid; l < slotLines; l += kNT) {
        const int q = ((l >> 7) << 6) + (l & 63), h = (l >> 6) & 1;
        const bool used = s0 + q < s1 && 2 * s.bufPack(s0 + q) + h < nlinesFull;
        if (!used) st16<kAuxFifo>(frs, (uint32_t)l * 16, (u32x4){0, sflag, 0, sflag});
      }
    }
    sendStep++;
  }

  // PRE (the pair kernel, runPair): pre[u] already holds this lane's source pack u of step 0
  template <bool REPOLL, bool PRE = false>
  __device__ void llFusedOp(const T* src, T* dst, const Shape s, const u32x4* pre = nullptr) {
    const int slotLines = uni(sc->llSlotLines);
    const int slotPacks = slotLines / 2;
    if (slotPacks > kNT * U) {  // several passes per step (NCCL_LL_BUFFSIZE raised): lockstep form
      [[clang::always_inline]] llOp<1, 1, 1, 1, 1>(src, dst, s);
      return;
    }
    constexpr int E = 8 / TS;
    const int nlinesFull = (s.n + E - 1) / E;
    const __amdgpu_buffer_rsrc_t srs = makeRsrc(src), drs = makeRsrc(dst);
    const bool vec = aligned16(src) && aligned16(dst);
    const int nsteps = s.npk > slotPacks ? (s.npk + slotPacks - 1) / slotPacks : 1;  // llOp: >= 1 step
    int B[U];
    bool act[U], two[U];
    u32x4 v[U];  // source of the step being received
    LAT_EV(11);
    waitSendCredit<kLLFifoSlots>();
    llStepPacks(s, slotPacks, nlinesFull, 0, B, act, two);
#pragma unroll
    for (int u = 0; u < U; u++)
      v[u] = !act[u] ? (u32x4){0, 0, 0, 0} : PRE ? pre[u] : loadPack(srs, vec, B[u], s.n);
    llSendLines(s, slotLines, nlinesFull, 0, min(s.npk, slotPacks), act, two, v);
    LAT_EV(12);
    for (int k = 0; k < nsteps; k++) {
      const int j = k + 1;
      const bool snd = j < nsteps;
      int Bs[U];
      bool as[U], ts[U];
      u32x4 vs[U];
      if (snd) {
        waitSendCredit<kLLFifoSlots>();
        llStepPacks(s, slotPacks, nlinesFull, j, Bs, as, ts);
#pragma unroll
        for (int u = 0; u < U; u++) vs[u] = as[u] ? loadPack(srs, vec, Bs[u], s.n) : (u32x4){0, 0, 0, 0};
      }
      llStepPacks(s, slotPacks, nlinesFull, k, B, act, two);
      const LLLine* rslot = rc->ll + (recvStep % kLLFifoSlots) * (uint64_t)slotLines;
      const uint32_t rflag = (uint32_t)(recvStep + 1) & llFlagMask;
      const void* la[2 * U];
      u32x4 ln[2 * U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int q = tid + u * kNT;
        la[2 * u] = act[u] ? rslot + llLineIdx(q, 0) : rslot;
        la[2 * u + 1] = two[u] ? rslot + llLineIdx(q, 1) : la[2 * u];
      }
      ldLines8(la, ln);
      // REPOLL (the exchange-set kernel, DESIGN.md §2 "LL polls"): every line of the lane
      // re-polled together while any is stale (one round trip for the late lines, not one per
      // pair); the per-pair loop below then finds every flag current.  32 MiB: 63.4 us against
      // 64.6 for per-pair polls, a wave-ballot spin 63.5 (profiles/r04i_lat.txt).  The general
      // small kernel keeps the per-pair polls: the loop's live lines spill its fp16 form
      if constexpr (REPOLL) {
        Spin spins;
        while (true) {
          bool stale = false;
#pragma unroll
          for (int u = 0; u < U; u++)
            stale |= act[u] && (ln[2 * u].y != rflag || ln[2 * u].w != rflag || ln[2 * u + 1].y != rflag ||
                                ln[2 * u + 1].w != rflag);
          if (!stale || spinAbort(spins)) break;
          ldLines8(la, ln);
        }
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        Spin spins;
        while (act[u] && (ln[2 * u].y != rflag || ln[2 * u].w != rflag || ln[2 * u + 1].y != rflag ||
                          ln[2 * u + 1].w != rflag)) {
          if (spinAbort(spins)) break;
          ldLines2(la[2 * u], la[2 * u + 1], ln[2 * u], ln[2 * u + 1]);
        }
        const u32x4 peer = {ln[2 * u].x, ln[2 * u].z, ln[2 * u + 1].x, ln[2 * u + 1].z};
        if (act[u]) storePack(drs, vec, B[u], s.n, F::pack(peer, v[u]));  // rrc: fn(peer, local)
      }
      LAT_EV(13);
      recvStep++;
      __syncthreads();
      if (tid == 0) atomicStoreSys(rc->remoteHead, recvStep);
      LAT_EV(14);
      if (snd) {
        llSendLines(s, slotLines, nlinesFull, j * slotPacks, min(s.npk, (j + 1) * slotPacks), as, ts, vs);
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = vs[u];
      }
    }
  }

  // ---------------------------------------------------------------- LL128, 1/2/4-byte types
  // One FIFO line per lane.  A unit of 3 packs (48 B) travels as 4 lines {12 B payload, 4-B
  // flag} (the same line contents as l16Step); lane (unit u, line j) carries payload bytes
  // [12j, 12j+12) of unit u in line 4u + j of the slot, so a wave's source loads (dwordx3), line
  // stores and line polls are each one contiguous 768 B / 1 KiB.  Units never straddle two
  // chunks of a split workgroup.  (8-byte elements straddle lanes: they take l16Step.)
  template <int RECV, int SEND, int SRC, int DST>
  __device__ void l16Op(const T* src, T* dst, const Shape s) {
    constexpr int UL = 4;  // lines per lane per pass (8 spills: 128 VGPRs)
    const int slotLines = uni(SEND ? sc->llSlotLines : rc->llSlotLines);
    const int unitsPerSlot = slotLines / 4;
    const bool contig = s.Lq == s.Q;  // the call's packs are one contiguous range
    const int upc = contig ? 1 : (s.Lq + 2) / 3;  // units per chunk segment (split)
    const int nUnits = contig ? (s.npk + 2) / 3 : (s.Lq > 0 ? (s.npk / s.Lq) * upc : 0);
    const int64_t nbytes = (int64_t)s.n * TS;
    __amdgpu_buffer_rsrc_t srs, drs, frs;
    if (SRC) srs = makeRsrc(src);
    if (DST) drs = makeRsrc(dst);
    const bool vec = (!SRC || aligned16(src)) && (!DST || aligned16(dst));
    int u0 = 0;
    do {
      const int u1 = nUnits - u0 < unitsPerSlot ? nUnits : u0 + unitsPerSlot;
      if (SEND) waitSendCredit<kLLFifoSlots>();
      LLLine* rslot = nullptr;
      uint32_t rflag = 0, sflag = 0;
      if (RECV) {
        rslot = rc->ll + (recvStep % kLLFifoSlots) * (uint64_t)rc->llSlotLines;
        rflag = (uint32_t)(recvStep + 1) & llFlagMask;
      }
      if (SEND) {
        frs = makeRsrc(sc->ll + (sendStep % kLLFifoSlots) * (uint64_t)sc->llSlotLines);
        sflag = (uint32_t)(sendStep + 1) & llFlagMask;
      }
      const int nLines = (u1 - u0) * 4;
      for (int base = tid; base < nLines; base += kNT * UL) {
        bool has[UL];
        uint32_t sb[UL];
        int vb[UL];
        u32x3 v[UL];
#pragma unroll
        for (int k = 0; k < UL; k++) {
          const int L = base + k * kNT;
          const int u = u0 + (L >> 2), j = L & 3;
          int bp, nv;
          if (contig) {
            bp = 3 * u;
            nv = s.npk - bp < 3 ? s.npk - bp : 3;
          } else {
            const int c = u / upc, uu = u - c * upc;
            bp = c * s.Q + s.q0 + 3 * uu;
            nv = s.Lq - 3 * uu < 3 ? s.Lq - 3 * uu : 3;
          }
          has[k] = L < nLines && 3 * j < 4 * nv;  // this line carries payload
          sb[k] = (uint32_t)(bp * 16 + 12 * j);
          int64_t lim = (int64_t)16 * nv - 12 * j;
          const int64_t left = nbytes - (int64_t)sb[k];
          lim = left < lim ? left : lim;
          vb[k] = has[k] ? (int)(lim < 0 ? 0 : (lim > 12 ? 12 : lim)) : 0;
          v[k] = (u32x3){0, 0, 0};
        }
        if (SRC) {
#pragma unroll
          for (int k = 0; k < UL; k++) {
            if (vb[k] == 12 && vec) v[k] = ld12<kAuxLocal>(srs, sb[k]);
            else if (vb[k] > 0) v[k] = loadBytes12(srs, sb[k], vb[k]);
          }
        }
        if (RECV) {
          const void* la[UL];
          u32x4 ln[UL];
#pragma unroll
          for (int k = 0; k < UL; k++) la[k] = rslot + (has[k] ? base + k * kNT : 0);
          ldLines4(la, ln);
#pragma unroll
          for (int k = 0; k < UL; k++) {
            Spin spins;
            while (has[k] && ln[k].w != rflag) {
              if (spinAbort(spins)) break;
              ldLine1(la[k], ln[k]);
            }
            const u32x4 peer = {ln[k].x, ln[k].y, ln[k].z, 0};
            if (SRC) {
              const u32x4 r = F::pack(peer, (u32x4){v[k].x, v[k].y, v[k].z, 0});
              v[k] = (u32x3){r.x, r.y, r.z};
            } else {
              v[k] = (u32x3){peer.x, peer.y, peer.z};
            }
          }
        }
        if (SEND) {
#pragma unroll
          for (int k = 0; k < UL; k++)
            if (has[k]) st16<kAuxFifo>(frs, (uint32_t)(base + k * kNT) * 16, (u32x4){v[k].x, v[k].y, v[k].z, sflag});
        }
        if (DST) {
#pragma unroll
          for (int k = 0; k < UL; k++) {
            if (vb[k] == 12 && vec) st12<kAuxLocal>(drs, sb[k], v[k]);
            else if (vb[k] > 0) storeBytes12(drs, sb[k], vb[k], v[k]);
          }
        }
      }
      if (SEND) {
        if ((sendStep & llCleanMask) == llCleanMask) {
          // LL cleanup (prims_ll.h:90-97): stamp every line of the slot that carries no payload
          for (int l = tid; l < slotLines; l += kNT) {
            const int u = u0 + (l >> 2), j = l & 3;
            bool used = false;
            if (l < nLines) {
              int nv;
              if (contig) nv = s.npk - 3 * u < 3 ? s.npk - 3 * u : 3;
              else {
                const int uu = u - (u / upc) * upc;
                nv = s.Lq - 3 * uu < 3 ? s.Lq - 3 * uu : 3;
              }
              used = 3 * j < 4 * nv;
            }
            if (!used) st16<kAuxFifo>(frs, (uint32_t)l * 16, (u32x4){0, sflag, 0, sflag});
          }
        }
        sendStep++;
      }
      if (RECV) {
        recvStep++;
        __syncthreads();
        if (tid == 0) atomicStoreSys(rc->remoteHead, recvStep);
      }
      u0 = u1;
    } while (u0 < nUnits);
  }

  // up to 12 bytes (whole elements) of a line's payload, zero-filled
  __device__ __forceinline__ u32x3 loadBytes12(__amdgpu_buffer_rsrc_t r, uint32_t off, int nb) {
    T e[12 / TS];
#pragma unroll
    for (int i = 0; i < 12 / TS; i++) {
      if (i * TS < nb) e[i] = ldElem<T>(r, off + i * TS);
      else __builtin_memset(&e[i], 0, TS);
    }
    u32x3 o;
    __builtin_memcpy(&o, e, 12);
    return o;
  }
  __device__ __forceinline__ void storeBytes12(__amdgpu_buffer_rsrc_t r, uint32_t off, int nb, u32x3 x) {
    T e[12 / TS];
    __builtin_memcpy(e, &x, 12);
#pragma unroll
    for (int i = 0; i < 12 / TS; i++)
      if (i * TS < nb) stElem<T>(r, off + i * TS, e[i]);
  }

  // one LL step: packs [s0, s1) of the call, U packs per lane per pass with all their loads and
  // line polls in flight together
  template <int RECV, int SEND, int SRC, int DST, int FUSED>
  __device__ void llStep(__amdgpu_buffer_rsrc_t srs, __amdgpu_buffer_rsrc_t drs,
                                         __amdgpu_buffer_rsrc_t frs, LLLine* rslot, uint32_t rflag,
                                         uint32_t sflag, bool vec, const Shape& s, int s0, int s1, int nlinesFull) {
    for (int base = tid; base < s1 - s0; base += kNT * U) {
      int B[U];
      bool act[U], two[U];
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int q = base + u * kNT;
        act[u] = q < s1 - s0;
        B[u] = act[u] ? s.bufPack(s0 + q) : 0;
        two[u] = act[u] && 2 * B[u] + 1 < nlinesFull;
        v[u] = (u32x4){0, 0, 0, 0};
      }
      if (SRC) {
#pragma unroll
        for (int u = 0; u < U; u++)
          if (act[u]) v[u] = loadPack(srs, vec, B[u], s.n);
        // preOp on data from the user's input (prims_ll.h:280; ring mode only, see PrePost)
        if constexpr (PP::kPre) {
#pragma unroll
          for (int u = 0; u < U; u++) v[u] = PP::pre(v[u], redArg);
        }
      }
      if (FUSED) {
        // the source goes out before this lane waits for the peer's lines: the peer's wait for
        // this step never depends on this workgroup's progress
#pragma unroll
        for (int u = 0; u < U; u++) {
          if (!act[u]) continue;
          const int q = base + u * kNT;
          st16<kAuxFifo>(frs, (uint32_t)llLineIdx(q, 0) * 16, (u32x4){v[u].x, sflag, v[u].y, sflag});
          if (two[u]) st16<kAuxFifo>(frs, (uint32_t)llLineIdx(q, 1) * 16, (u32x4){v[u].z, sflag, v[u].w, sflag});
        }
      }
      if (RECV) {
        const void* la[2 * U];
        u32x4 ln[2 * U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const int q = base + u * kNT;
          la[2 * u] = act[u] ? rslot + llLineIdx(q, 0) : rslot;
          la[2 * u + 1] = two[u] ? rslot + llLineIdx(q, 1) : la[2 * u];
        }
        ldLines8(la, ln);
#pragma unroll
        for (int u = 0; u < U; u++) {
          Spin spins;
          while (act[u] && (ln[2 * u].y != rflag || ln[2 * u].w != rflag || ln[2 * u + 1].y != rflag ||
                            ln[2 * u + 1].w != rflag)) {
            if (spinAbort(spins)) break;
            ldLines2(la[2 * u], la[2 * u + 1], ln[2 * u], ln[2 * u + 1]);
          }
          const u32x4 peer = {ln[2 * u].x, ln[2 * u].z, ln[2 * u + 1].x, ln[2 * u + 1].z};
          v[u] = SRC ? F::pack(peer, v[u]) : peer;
        }
        // postOp on the final reduction of the ring (rrcs / rrc, all_reduce.h:84,
        // reduce_scatter.h:65: the only receive-reduce transfers with an output)
        if constexpr (PP::kPost && SRC && DST) {
#pragma unroll
          for (int u = 0; u < U; u++) v[u] = PP::post(v[u], redArg);
        }
      }
      if (SEND && !FUSED) {
#pragma unroll
        for (int u = 0; u < U; u++) {
          if (!act[u]) continue;
          const int q = base + u * kNT;
          st16<kAuxFifo>(frs, (uint32_t)llLineIdx(q, 0) * 16, (u32x4){v[u].x, sflag, v[u].y, sflag});
          if (two[u]) st16<kAuxFifo>(frs, (uint32_t)llLineIdx(q, 1) * 16, (u32x4){v[u].z, sflag, v[u].w, sflag});
        }
      }
      if (DST) {
#pragma unroll
        for (int u = 0; u < U; u++)
          if (act[u]) storePack(drs, vec, B[u], s.n, v[u]);
      }
    }
  }

  // one LL128 step: units of 3 packs / 4 lines, two units per lane per pass (8 lines in flight)
  template <int RECV, int SEND, int SRC, int DST>
  __device__ void l16Step(__amdgpu_buffer_rsrc_t srs, __amdgpu_buffer_rsrc_t drs,
                                          __amdgpu_buffer_rsrc_t frs, LLLine* rslot, uint32_t rflag,
                                          uint32_t sflag, bool vec, const Shape& s, int s0, int s1) {
    constexpr int UU = 2;
    const int units = (s1 - s0 + 2) / 3;
    for (int base = tid; base < units; base += kNT * UU) {
      int nv[UU], B[UU][3];
      u32x4 v[UU][3];
#pragma unroll
      for (int k = 0; k < UU; k++) {
        const int u = base + k * kNT;
        const int rem = u < units ? s1 - s0 - 3 * u : 0;
        nv[k] = rem < 3 ? rem : 3;
#pragma unroll
        for (int j = 0; j < 3; j++) {
          B[k][j] = j < nv[k] ? s.bufPack(s0 + 3 * u + j) : 0;
          v[k][j] = (u32x4){0, 0, 0, 0};
        }
      }
      if (SRC) {
#pragma unroll
        for (int k = 0; k < UU; k++)
#pragma unroll
          for (int j = 0; j < 3; j++)
            if (j < nv[k]) v[k][j] = loadPack(srs, vec, B[k][j], s.n);
      }
      if (RECV) {
        const void* la[4 * UU];
        u32x4 ln[4 * UU];
#pragma unroll
        for (int k = 0; k < UU; k++) {
          const int u = base + k * kNT;
          const int nl = nv[k] > 0 ? l16Lines(nv[k]) : 0;
#pragma unroll
          for (int j = 0; j < 4; j++)
            la[4 * k + j] = j < nl ? (const void*)(rslot + l16LineIdx(u, j)) : (const void*)rslot;
        }
        ldLines8(la, ln);
#pragma unroll
        for (int k = 0; k < UU; k++) {
          const int nl = nv[k] > 0 ? l16Lines(nv[k]) : 0;
          Spin spins;
          while ((nl > 0 && ln[4 * k].w != rflag) || (nl > 1 && ln[4 * k + 1].w != rflag) ||
                 (nl > 2 && ln[4 * k + 2].w != rflag) || (nl > 3 && ln[4 * k + 3].w != rflag)) {
            if (spinAbort(spins)) break;
            ldLines2(la[4 * k], la[4 * k + 1], ln[4 * k], ln[4 * k + 1]);
            ldLines2(la[4 * k + 2], la[4 * k + 3], ln[4 * k + 2], ln[4 * k + 3]);
          }
          // 12 payload dwords of the unit -> 3 packs
          const u32x4 p0 = {ln[4 * k].x, ln[4 * k].y, ln[4 * k].z, ln[4 * k + 1].x};
          const u32x4 p1 = {ln[4 * k + 1].y, ln[4 * k + 1].z, ln[4 * k + 2].x, ln[4 * k + 2].y};
          const u32x4 p2 = {ln[4 * k + 2].z, ln[4 * k + 3].x, ln[4 * k + 3].y, ln[4 * k + 3].z};
          v[k][0] = SRC ? F::pack(p0, v[k][0]) : p0;
          v[k][1] = SRC ? F::pack(p1, v[k][1]) : p1;
          v[k][2] = SRC ? F::pack(p2, v[k][2]) : p2;
        }
      }
      if (SEND) {
#pragma unroll
        for (int k = 0; k < UU; k++) {
          if (nv[k] == 0) continue;
          const int u = base + k * kNT;
          const int nl = l16Lines(nv[k]);
          st16<kAuxFifo>(frs, (uint32_t)l16LineIdx(u, 0) * 16, (u32x4){v[k][0].x, v[k][0].y, v[k][0].z, sflag});
          st16<kAuxFifo>(frs, (uint32_t)l16LineIdx(u, 1) * 16, (u32x4){v[k][0].w, v[k][1].x, v[k][1].y, sflag});
          if (nl > 2)
            st16<kAuxFifo>(frs, (uint32_t)l16LineIdx(u, 2) * 16, (u32x4){v[k][1].z, v[k][1].w, v[k][2].x, sflag});
          if (nl > 3)
            st16<kAuxFifo>(frs, (uint32_t)l16LineIdx(u, 3) * 16, (u32x4){v[k][2].y, v[k][2].z, v[k][2].w, sflag});
        }
      }
      if (DST) {
#pragma unroll
        for (int k = 0; k < UU; k++)
#pragma unroll
          for (int j = 0; j < 3; j++)
            if (j < nv[k]) storePack(drs, vec, B[k][j], s.n, v[k][j]);
      }
    }
  }

  // ---------------------------------------------------------------- Simple protocol
  template <int RECV, int SEND, int SRC, int DST>
  __device__ void simpleOp(const T* src, T* dst, const Shape s) {
    const int slotBytes = uni(SEND ? sc->simpleSlotBytes : rc->simpleSlotBytes);
    const int slicePacks = slotBytes / 16;
    __amdgpu_buffer_rsrc_t srs, drs, rrs, frs;
    if (SRC) srs = makeRsrc(src);
    if (DST) drs = makeRsrc(dst);
    const bool vec = (!SRC || aligned16(src)) && (!DST || aligned16(dst));
    for (int s0 = 0; s0 < s.npk; s0 += slicePacks) {
      const int s1 = s.npk - s0 < slicePacks ? s.npk : s0 + slicePacks;
      if (RECV) waitRecvTail();
      if (SEND) waitSendCredit<kFifoSteps>();
      __syncthreads();
      if (RECV) rrs = makeRsrc(rc->simple + (recvStep % kFifoSteps) * (uint64_t)slotBytes);
      if (SEND) frs = makeRsrc(sc->simple + (sendStep % kFifoSteps) * (uint64_t)slotBytes);
      // packs per lane per pass: copies (one source: the FIFO or the input) keep UC in flight,
      // reductions (both) U
      constexpr int UU = RECV && SRC ? U : kSimpleCopyU;
      for (int base = s0 + tid; base < s1; base += kNT * UU) {
        int B[UU];
        bool act[UU];
        u32x4 v[UU], peer[UU];
#pragma unroll
        for (int u = 0; u < UU; u++) {
          const int p = base + u * kNT;
          act[u] = p < s1;
          B[u] = act[u] ? s.bufPack(p) : 0;
          v[u] = peer[u] = (u32x4){0, 0, 0, 0};
        }
        if (SRC) {
#pragma unroll
          for (int u = 0; u < UU; u++)
            if (act[u]) v[u] = loadPack(srs, vec, B[u], s.n);
          if constexpr (PP::kPre) {  // PreOpN = 1: the local input (prims_simple.h:209-211)
#pragma unroll
            for (int u = 0; u < UU; u++) v[u] = PP::pre(v[u], redArg);
          }
        }
        if (RECV) {
#pragma unroll
          for (int u = 0; u < UU; u++)
            if (act[u]) peer[u] = ld16<kAuxFifo>(rrs, (uint32_t)(base + u * kNT - s0) * 16);
#pragma unroll
          for (int u = 0; u < UU; u++) v[u] = SRC ? F::pack(v[u], peer[u]) : peer[u];
          if constexpr (PP::kPost && SRC && DST) {
#pragma unroll
            for (int u = 0; u < UU; u++) v[u] = PP::post(v[u], redArg);
          }
        }
#pragma unroll
        for (int u = 0; u < UU; u++) {
          if (!act[u]) continue;
          if (SEND) st16<kAuxFifo>(frs, (uint32_t)(base + u * kNT - s0) * 16, v[u]);
          if (DST) storePack(drs, vec, B[u], s.n, v[u]);
        }
      }
      // Hand-off (waitRecvTail): every lane's FIFO stores -- and its loads of the slot it frees --
      // drain, the workgroup barrier, then one lane posts the tail (the data) and the head (the
      // freed slot) with sc0 sc1 stores.  Towards another GPU a system-scope release comes first
      // (the reference's __threadfence_system before postPeer, prims_simple.h:122-128,218).
      drainStores();
      __syncthreads();
      if (tid == 0) {
        const int rem = (SEND ? sc->remote : 0) | (RECV ? rc->remote : 0);
        if (rem & 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        else if (rem == 2) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        if (SEND) atomicStoreSys(sc->remoteTail, sendStep + 1);
        if (RECV) atomicStoreSys(rc->remoteHead, recvStep + 1);
      }
      if (SEND) sendStep++;
      if (RECV) recvStep++;
    }
  }

  template <int RECV, int SEND, int SRC, int DST>
  __device__ __forceinline__ void op(const T* src, T* dst, const Shape s) {
    if constexpr (PROTO == pSimple) simpleOp<RECV, SEND, SRC, DST>(src, dst, s);
    else if constexpr (PROTO == pLL128 && TS <= 4) l16Op<RECV, SEND, SRC, DST>(src, dst, s);
    else llOp<RECV, SEND, SRC, DST>(src, dst, s);  // LL, and LL128 of 8-byte types
  }

  // ---------------------------------------------------------------- local ops
  __device__ __forceinline__ void localCopy(const T* src, T* dst, const Shape s) {
    __amdgpu_buffer_rsrc_t srs = makeRsrc(src), drs = makeRsrc(dst);
    const bool vec = aligned16(src) && aligned16(dst);
    for (int base = tid; base < s.npk; base += kNT * U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++)
        if (base + u * kNT < s.npk) v[u] = loadPack(srs, vec, s.bufPack(base + u * kNT), s.n);
#pragma unroll
      for (int u = 0; u < U; u++)
        if (base + u * kNT < s.npk) storePack(drs, vec, s.bufPack(base + u * kNT), s.n, v[u]);
    }
  }

  // Source r of the fused reduction starts at srcBase + chunkOff + reds[r] * sizePer (reds: chunk
  // indices in LDS, at most MSCCL_MAX_REDUCE_FUSION = 16).  The per-element path is chosen on the whole call's element count, as in the reference.
  __device__ __forceinline__ void reduce(const T* srcBase, const int16_t* reds, int64_t chunkOff, int64_t sizePer, int nsrc, T* dst,
                         const Shape s) {
    if (s.n < refNthreads) {
      // per-element path, d first: o = fn(s_r, o) (msccl_interpreter.h:157-170)
      __amdgpu_buffer_rsrc_t drs = makeRsrc(dst);
      // all (at most MSCCL_MAX_REDUCE_FUSION) sources are loaded before the fold, so the
      // element costs one memory round trip instead of one per source
      for (int k = tid; k < s.npk * PE; k += kNT) {
        const int e = s.bufPack(k / PE) * PE + (k % PE);
        if (e >= s.n) continue;
        T o = ldElem<T>(drs, (uint32_t)e * TS);
        T x[16];
#pragma unroll
        for (int r = 0; r < 16; r++)
          if (r < nsrc) x[r] = ldElem<T>(makeRsrc(srcBase + chunkOff + reds[r] * sizePer), (uint32_t)e * TS);
#pragma unroll
        for (int r = 0; r < 16; r++)
          if (r < nsrc) o = F::elem(x[r], o);
        stElem<T>(drs, (uint32_t)e * TS, o);
      }
      return;
    }
    __amdgpu_buffer_rsrc_t drs = makeRsrc(dst);
    bool vec = aligned16(dst);
    for (int r = 0; r < nsrc; r++) vec = vec && aligned16(srcBase + chunkOff + reds[r] * sizePer);
    for (int base = tid; base < s.npk; base += kNT * U) {
      int B[U];
      bool act[U];
      u32x4 d[U], acc[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        act[u] = base + u * kNT < s.npk;
        B[u] = act[u] ? s.bufPack(base + u * kNT) : 0;
        d[u] = acc[u] = (u32x4){0, 0, 0, 0};
        if (act[u]) d[u] = loadPack(drs, vec, B[u], s.n);
      }
      for (int r = 0; r < nsrc; r++) {
        const __amdgpu_buffer_rsrc_t rs = makeRsrc(srcBase + chunkOff + reds[r] * sizePer);
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; u++) x[u] = act[u] ? loadPack(rs, vec, B[u], s.n) : (u32x4){0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; u++) {
          if constexpr (PROTO == pSimple) acc[u] = r == 0 ? x[u] : F::pack(acc[u], x[u]);  // (s0(+)s1..)(+)d
          else if constexpr (PROTO == pLL128) acc[u] = F::pack(x[u], r == 0 ? d[u] : acc[u]);  // fn(s, acc)
          else acc[u] = F::pack(r == 0 ? d[u] : acc[u], x[u]);                             // fn(acc, s)
        }
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        if (!act[u]) continue;
        if constexpr (PROTO == pSimple) acc[u] = F::pack(acc[u], d[u]);
        storePack(drs, vec, B[u], s.n, acc[u]);
      }
    }
  }

  // ---------------------------------------------------------------- launch prologue / epilogue
  // Prologue: one memory round trip.  The image (header + program), both connection records
  // and the launch epoch sit at addresses known from the block index, so all of them are in
  // flight together: the image by lane i for unit i (waves 0-5, kMaxImage16 units), the two
  // records by lanes 448-455 (wave 7), the epoch by lane 384 (wave 6).  No wave issues two of
  // them: a wave's LDS store waits for its load, and a second load behind it would be a second
  // round trip (it was, for the image and the send record both in wave 0).  Returns the launch
  // epoch (workIndex).
  __device__ __forceinline__ uint64_t prologue(const RankWork& w, int bid, int sub, DevTbHeader& hd) {
    tid = threadIdx.x;
    comm = w.comm;
    refNthreads = w.refNthreads;
    timeoutTicks = w.timeoutTicks;
    llFlagMask = w.llFlagMask;
    llCleanMask = w.llCleanMask;
    const int slot = bid * w.maxSplit + sub;      // flag / epoch / trace slot of this workgroup
    const int cslot = bid * w.connSplit + sub;    // its connection records
    {
      static_assert(kMaxImage16 <= 384, "image units must stay in waves 0-5");
      const u32x4* gimg = (const u32x4*)(w.images + (size_t)bid * w.tbStride);
      const int nU = w.tbStride >> 4;
      if (tid < nU) sh->img[tid] = gimg[tid];
      if (tid >= 448 && tid < 456) {
        const int j = tid - 448;
        const u32x4* src = j < 4 ? (const u32x4*)(w.send + cslot) + j : (const u32x4*)(w.recv + cslot) + (j - 4);
        u32x4* dst = j < 4 ? (u32x4*)&sh->sconn + j : (u32x4*)&sh->rconn + (j - 4);
        *dst = *src;
      }
      if (tid == 384) {
        sh->aborted = 0;
        sh->epoch = atomicLoadAgent(w.epochs + slot);
      }
    }
    __syncthreads();
    {
      u32x4 raw = sh->img[0];
      raw = (u32x4){uni(raw.x), uni(raw.y), uni(raw.z), uni(raw.w)};
      __builtin_memcpy(&hd, &raw, sizeof(hd));
    }
    tr = (const DevTransfer*)&sh->img[1];
    depBid = (const int16_t*)(tr + hd.nsteps);
    depStep = depBid + hd.ndeps;
    red = depStep + hd.ndeps;
    scG = hd.hasSend ? w.send + cslot : nullptr;
    rcG = hd.hasRecv ? w.recv + cslot : nullptr;
    sc = scG ? &sh->sconn : nullptr;
    rc = rcG ? &sh->rconn : nullptr;
    sendStep = scG ? uni(sh->sconn.step) : 0;
    recvStep = rcG ? uni(sh->rconn.step) : 0;
    headSeen = scG ? uni(sh->sconn.headSeen) : 0;
    tailSeen = rcG ? uni(sh->rconn.tailSeen) : 0;
    return uni(sh->epoch);  // COMPUTE_FLAG's workIndex (msccl_interpreter.h:14-16)
  }

  // Epilogue: persist the connection state and advance this slot's epoch, plus the epoch of
  // every slot of the schedule's range this launch does not run (DevComm::epochs): the subs
  // [split, maxSplit) of each launched tb (by that tb's sub 0), and the slots of the tbs beyond
  // this launch's, [nTb * maxSplit, epochSlots) (ring / tree channels not used by this call),
  // dealt over the launch's workgroups.  An MSCCL schedule always runs all its tbs: nothing there.
  __device__ __forceinline__ void epilogue(const RankWork& w, int bid, int sub, uint64_t workIndex) {
    const int split = w.split, maxSplit = w.maxSplit;
    __syncthreads();
    if (tid == 0) {
      if (scG) {
        scG->step = sendStep;
        scG->headSeen = headSeen;
      }
      if (rcG) {
        rcG->step = recvStep;
        rcG->tailSeen = tailSeen;
      }
      atomicStoreAgent(w.epochs + bid * maxSplit + sub, workIndex + 1);
    }
    const int launched = w.nBlocks, nTb = launched / split, g = bid * split + sub;
    if (sub == 0 && tid < maxSplit - split) atomicStoreAgent(w.epochs + bid * maxSplit + split + tid, workIndex + 1);
    for (int j = nTb * maxSplit + g + tid * launched; j < w.epochSlots; j += kNT * launched)
      atomicStoreAgent(w.epochs + j, workIndex + 1);
  }

  // Wait for the same positions of the thread blocks transfer t depends on
  // (msccl_interpreter.h:123-140)
  __device__ __forceinline__ void waitDeps(const DevTransfer& t, const uint64_t* flags, uint64_t workIndex,
                                           uint64_t iter, int sub, int maxSplit) {
    if (tid < t.numDeps) {
      const int db = depBid[t.depPtr + tid];
      const uint64_t goal = computeFlag(workIndex, iter, (uint64_t)depStep[t.depPtr + tid]);
      Spin spins;
      while (true) {
        uint64_t cur = atomicLoadAgent(flags + ((size_t)db * maxSplit + sub) * kFlagStride);
        if (cur >= goal && (cur >> 24) == workIndex) break;
        if (spinAbort(spins)) break;
      }
    }
    __syncthreads();
  }

  // One primitive call of transfer t; false for MSCCL_RES_ADD / unknown types (the tb ends,
  // msccl_interpreter.h:195-196).  `reOff` is the chunk offset of a fused reduction's sources.
  template <bool FUSE, int SET = kSetAll>
  __device__ __forceinline__ bool exec(const DevTransfer& t, T* srcP, T* dstP, int64_t srcoff, int64_t dstoff,
                                       int64_t reOff, int64_t sizePer, const Shape& s) {
    if constexpr (SET == kSetExchange) {
      // the exchange kernels (devcomm.h: kSetExchange): the pair exchange's transfers only
      switch (t.type) {
        case tSend: op<0, 1, 1, 0>(srcP + srcoff, nullptr, s); __syncthreads(); break;
        case tRRC: op<1, 0, 1, 1>(srcP + srcoff, dstP + dstoff, s); break;
        case tSendRrc:
          if constexpr (FUSE && PROTO == pLL && OP <= 3) [[clang::always_inline]] llFusedOp<true>(srcP + srcoff, dstP + dstoff, s);
          break;
        default: return false;
      }
      return true;
    }
    switch (t.type) {
      case tSend: op<0, 1, 1, 0>(srcP + srcoff, nullptr, s); __syncthreads(); break;
      case tRecv: op<1, 0, 0, 1>(nullptr, dstP + dstoff, s); break;
      case tRCS: op<1, 1, 0, 1>(nullptr, dstP + dstoff, s); break;
      case tRRS: op<1, 1, 1, 0>(srcP + srcoff, nullptr, s); break;
      case tRRC: op<1, 0, 1, 1>(srcP + srcoff, dstP + dstoff, s); break;
      case tRRCS: op<1, 1, 1, 1>(srcP + srcoff, dstP + dstoff, s); break;
      case tCpy: localCopy(srcP + srcoff, dstP + dstoff, s); __syncthreads(); break;
      case tCopySend: op<0, 1, 1, 1>(srcP + srcoff, dstP + dstoff, s); __syncthreads(); break;
      case tSendRrc:  // LL only (run / runSmall turn it into tSend otherwise); dst from the rrc
        if constexpr (FUSE && PROTO == pLL && OP <= 3) {  // MSCCL schedules run Sum..Min only
          // inlined like the other primitive calls (a call frame costs scratch and SGPR spills)
          [[clang::always_inline]] llFusedOp<false>(srcP + srcoff, dstP + dstoff, s);
        }
        break;
      case tRe: reduce(srcP, red + t.redPtr, reOff, sizePer, t.numReds, dstP + dstoff, s); __syncthreads(); break;
      default: return false;
    }
    return true;
  }

  static __device__ __forceinline__ DevTransfer loadTransfer(const DevTransfer* p) {
    DevTransfer t;
    u32x4 raw = *(const u32x4*)p;
    raw = (u32x4){uni(raw.x), uni(raw.y), uni(raw.z), uni(raw.w)};
    __builtin_memcpy(&t, &raw, sizeof(t));
    return t;
  }

  // a tSendRrc transfer runs fused with LL in mscclSmallKernel (FUSE) when both FIFO slot sizes
  // agree (the two ends then cut the same steps); otherwise, and always in the general kernel
  // (trace, NPKit, uneven passes: its register budget has no room for the fused pipeline), as
  // its s followed by its rrc, which a fused peer interoperates with (transport.cc: fusableTbs)
  template <bool FUSE>
  __device__ __forceinline__ bool fuseable(const DevTransfer& t) const {
    if constexpr (!FUSE || PROTO != pLL || OP > 3) return false;
    return t.type == tSendRrc && uni(sc->llSlotLines) == uni(rc->llSlotLines);
  }

  __device__ __forceinline__ void publishFlag(uint64_t* flags, int slot, uint64_t workIndex, uint64_t iter, int step) {
    drainStores();
    __syncthreads();
    if (tid == 0) atomicStoreAgent(flags + (size_t)slot * kFlagStride, computeFlag(workIndex, iter, step));
  }

  // ---------------------------------------------------------------- the interpreter loop
  // Nothing before the prologue waits on a kernel argument or reads the clock: a stamp at entry
  // (s_memrealtime is a scalar-memory op: the first wait for a kernel argument waits for it too)
  // or a branch on an argument delayed the prologue's loads of every launch (the fold kernel:
  // 0.5 us, profiles/r04c_lat.txt); the clock is read after the prologue, and only when traced.
  __device__ __forceinline__ void run(const RankWork& w, int bid, int sub) {
    const int split = w.split;
    const int maxSplit = w.maxSplit;
    const int slot = bid * maxSplit + sub;
    DevTbHeader hd;
    const uint64_t workIndex = prologue(w, bid, sub, hd);
    t0 = w.trace != nullptr || w.npkit != nullptr ? __builtin_amdgcn_s_memrealtime() : 0;
    redArg = w.redOpArg;
    if (w.redOpArgIsPtr) {  // ncclScalarDevice: the scale lives in device memory (enqueue.cc:1549-1557)
      T x;
      __builtin_memcpy(&x, (const void*)w.redOpArg, sizeof(T));
      redArg = 0;
      __builtin_memcpy(&redArg, &x, sizeof(T));
      redArg = uni(redArg);
    }
    trace = w.trace ? w.trace + (size_t)slot * w.traceEvents : nullptr;
    nev = 1;
    maxEv = w.traceEvents;
    ev(kEvSetup, 0, 0);
    nkBuf = nullptr;
    if (w.npkit != nullptr && sub == 0 && bid < kNpkitDevBuffers) {
      // NPKIT_GPU_SYNC_TIME(bid, tid) (msccl_interpreter.h:88): the host time of this launch
      // start, then the GPU clock it corresponds to
      const NpkitLog* lg = w.npkit;
      nkCap = lg->cap;
      nkBuf = lg->events + (size_t)bid * nkCap;
      nkHeadG = lg->heads + bid;
      nkHead = uni(*nkHeadG);
      nk(NPKIT_EVENT_TIME_SYNC_CPU, 0, (uint64_t)(npkitTicksToNs(t0, lg->clockKHz) + lg->cpuOffsetNs));
      nk(NPKIT_EVENT_TIME_SYNC_GPU, 0, t0);
    }

    T* thisInput = (T*)w.sendbuff;
    T* thisOutput = (T*)w.recvbuff;
    T* thisScratch = (T*)w.scratch;
    const int64_t sizePer = w.sizePerChunk;
    const int64_t chunkSize = w.chunkSize;
    const int mac = w.maxAllowedCount;
    uint64_t* flags = w.flags;
    bool stop = false;

    const int64_t merge = w.merge;
    // ring fallback mode (w.ringColl != kRingNone): the reference's runRing loop over gridOffset
    const int ringColl = w.ringColl;
    // the tree runs two workgroups per channel: channel = bid / 2 (transport.cc: treePeers)
    const bool tree = ringColl == kTreeAllReduce;
    const int64_t ringSize = w.ringSize, nr = w.ringRanks, C = tree ? w.nBlocks / 2 : w.nBlocks;
    const int64_t chan = tree ? bid >> 1 : bid;
    int64_t nelemGrid = 0;
    for (int64_t grid = 0, iter = 0; grid < (ringColl ? ringSize : sizePer) && !stop; grid += nelemGrid, iter++) {
      int64_t real;
      int64_t ringCo = 0;  // ReduceScatter / AllGather chunkOffset
      if (ringColl) {
        const int64_t loop = ringColl == kRingAllReduce ? C * nr * chunkSize : C * chunkSize;
        const int64_t left = ringSize - grid;
        if (tree) {
          real = chunkSize;  // host-final chunk (runTreeUpDown / runTreeSplit: all_reduce.h:121-122)
        } else if (ringColl == kRingAllReduce) {
          if constexpr (PROTO == pSimple) {  // all_reduce.h:43-46
            real = (left + C * nr - 1) / (C * nr);
            real = real < chunkSize ? real : chunkSize;
            real = (real + w.minChunk - 1) / w.minChunk * w.minChunk;
          } else {                           // all_reduce.h:48
            real = (left + C * nr * w.minChunk - 1) / (C * nr * w.minChunk) * w.minChunk;
            real = real < chunkSize ? real : chunkSize;
          }
        } else {
          if constexpr (PROTO == pSimple) {  // reduce_scatter.h:33-36, all_gather.h:35-38
            real = (left + C - 1) / C;
            real = real < chunkSize ? real : chunkSize;
            real = (real + w.minChunk - 1) / w.minChunk * w.minChunk;
          } else {                           // reduce_scatter.h:37-38 (lastChunkSize)
            real = left < loop ? w.ringLastChunk : chunkSize;
          }
        }
        real = (int)real;
        ringCo = grid + chan * real;
        nelemGrid = loop;
      } else if constexpr (PROTO == pSimple) {
        real = sizePer - grid < chunkSize ? sizePer - grid : chunkSize;
        real = divNonNeg(real + w.minChunk - 1, w.minChunk) * w.minChunk;
      } else {
        int64_t rem = divNonNeg(sizePer - grid + w.minChunk - 1, w.minChunk) * w.minChunk;
        real = rem < chunkSize ? rem : chunkSize;
      }
      int nelem = 0;
      if (!ringColl) {
        real = (int)real;
        nelem = (int)(real < sizePer - grid ? real : sizePer - grid);
        if (nelem == chunkSize && merge > 1) {
          // run up to `merge` consecutive full iterations as one (enqueue.cc: makeWork)
          const int64_t full = (sizePer - grid) / chunkSize;
          nelem = (int)(chunkSize * (full < merge ? full : merge));
        }
        nelemGrid = nelem;
      }
      // this workgroup's positions inside every chunk of this iteration (nelem % PE == 0
      // whenever split > 1: the host sets split = 1 otherwise)
      const int Qc = (nelem + PE - 1) / PE;
      const int q0 = (int)divNonNeg((int64_t)Qc * sub, split), q1 = (int)divNonNeg((int64_t)Qc * (sub + 1), split);
      int step = 0;
      for (int i = 0; i < hd.nsteps; i++) {
        DevTransfer t = loadTransfer(&tr[i]);
        const bool fused = fuseable<false>(t);
        if (t.type == tSendRrc && !fused) t.type = tSend;
        const bool sendCpy = t.type == tSendCpy;  // s + cpy as one copy-send (dst: the cpy's)
        if (sendCpy) t.type = tCopySend;
        const DevTransfer td = fused || sendCpy ? loadTransfer(&tr[i + 1]) : t;  // output buffer
        if (t.numDeps > 0) {
          nk(NPKIT_EVENT_DEP_CHECK_ENTRY, t.numDeps);
          waitDeps(t, flags, workIndex, iter, sub, maxSplit);
          nk(NPKIT_EVENT_DEP_CHECK_EXIT, t.numDeps);
          step += t.numDeps - 1;
          ev(kEvDepWait, (uint16_t)i, 0);
        }
        T* srcP = t.srcbuf == 0 ? thisInput : (t.srcbuf == 1 ? thisOutput : thisScratch);
        T* dstP = td.dstbuf == 0 ? thisInput : (td.dstbuf == 1 ? thisOutput : thisScratch);
        // maxAllowedCount keeps one reference primitive call within one FIFO step
        // (enqueue.cc:700-711); these primitives cut calls into FIFO steps themselves, so when the
        // iteration covers whole chunks (consecutive chunks are contiguous) a transfer's chunks
        // move as one call.  Not for `re`: its per-element path depends on the call's size.
        // The rule depends only on (nelem, count), which the two ends of a connection share, so
        // a sender and its receiver cut the same calls and hence the same FIFO steps (a sender
        // splitting a transfer its receiver moves whole would misalign the steps whenever a call
        // is not a whole number of slots).  Calls stay within kMaxRunSlots slots per
        // sub-connection, and so far below the 2 GiB reach of a buffer descriptor.
        // (runSmall applies the same rule: the two ends may run different kernels.)
        int macT = (t.type != tRe && !ringColl && nelem == sizePer &&
                    (int64_t)nelem * t.count <= w.maxOpElems) ? t.count : mac;
        if ((int64_t)nelem * TS * macT > (int64_t)0x7fffff00) {
          // buffer descriptors address 2^31 - 1 bytes from a call's base (makeRsrc)
          const int64_t reach = (int64_t)0x7fffff00 / ((int64_t)nelem * TS);
          macT = reach < 1 ? 1 : (int)reach;
        }
        for (int c = 0; c < t.count; c += macT) {
          int64_t srcoff = grid + (int64_t)(t.srcoff + c) * sizePer;
          int64_t dstoff = grid + (int64_t)(td.dstoff + c) * sizePer;
          const int thisCount = macT < t.count - c ? macT : t.count - c;
          Shape s;
          s.n = nelem * thisCount;
          if (ringColl) {
            // offsets are chunk indices (AllReduce, all_reduce.h:51-56) or rank indices
            // (ReduceScatter / AllGather, -1 = chunkOffset alone); nelem = min(real, size - offset)
            int64_t lim;
            if (ringColl == kRingAllReduce) {
              const int64_t ci = t.srcoff >= 0 ? t.srcoff : t.dstoff;
              if constexpr (PROTO == pSimple) srcoff = grid + bid * nr * real + ci * real;
              else srcoff = grid + (ci * C + bid) * real;
              dstoff = srcoff;
              lim = srcoff;
            } else {
              srcoff = ringCo + (t.srcoff >= 0 ? (int64_t)t.srcoff * ringSize : 0);
              dstoff = ringCo + (t.dstoff >= 0 ? (int64_t)t.dstoff * ringSize : 0);
              lim = ringCo;
            }
            const int64_t ne = ringSize - lim < real ? ringSize - lim : real;
            s.n = ne > 0 ? (int)ne : 0;
          }
          if (split == 1) {
            s.Q = (s.n + PE - 1) / PE;
            s.q0 = 0;
            s.Lq = s.Q;
            s.npk = s.Q;
          } else {
            s.Q = Qc;
            s.q0 = q0;
            s.Lq = q1 - q0;
            s.npk = thisCount * s.Lq;
          }
          if (trace != nullptr && tid == 0) sh->waitTail = sh->waitHead = 0;
          ev(kEvPrimBegin, (uint16_t)i, ((uint32_t)t.type << 24) | (uint32_t)min(s.npk * PE, 0xFFFFFF));
          nk(nkPrim(t.type), (uint64_t)s.n * TS);
          if (!exec<false>(t, srcP, dstP, srcoff, dstoff, grid + (int64_t)c * sizePer, sizePer, s)) {
            stop = true;
            break;
          }
          nk(nkPrim(t.type) + 1, (uint64_t)s.n * TS);
          if (t.type == tRe && c == 0) step += t.numReds - 1;
          // arg: ticks waited for the Simple tail (high half) and for send credit (low half)
          ev(kEvPrimEnd, (uint16_t)i, trace != nullptr && tid == 0 ? ((uint32_t)sh->waitTail << 16) | sh->waitHead : 0);
        }
        if (stop) break;
        if (fused || sendCpy) {  // the s published nothing (transport.cc); the second transfer's flag below
          step++;
          i++;
          t = td;
        }
        if (t.hasDep) publishFlag(flags, slot, workIndex, iter, step);
        step++;
      }
    }
    epilogue(w, bid, sub, workIndex);
    if (nkBuf != nullptr && tid == 0) *nkHeadG = nkHead;
    ev(kEvEnd, 0, 0);
    if (trace != nullptr && tid == 0) {
      TraceEvent h;
      h.ts = t0;
      h.type = kEvHeader;
      h.step = (uint16_t)nev;
      h.arg = (uint32_t)workIndex;
      trace[0] = h;
    }
  }

  // pack B of block `blk` (n elements each) of a buffer of consecutive blocks
  __device__ __forceinline__ u32x4 loadBlockPack(const T* base, int blk, int n, int B) {
    const T* b = base + (size_t)blk * n;
    return loadPack(makeRsrc(b), aligned16(b), B, n);
  }
  __device__ __forceinline__ void storeBlockPack(T* base, int blk, int n, int B, u32x4 x) {
    T* b = base + (size_t)blk * n;
    storePack(makeRsrc(b), aligned16(b), B, n, x);
  }

  // ---------------------------------------------------------------- the flat tree (mscclFoldKernel)
  // The flat tree's one-hop AllReduce (transport.cc: ringUpload, plan.cc: makeFlatTreePlan), one
  // workgroup per 512 packs of the call (RankWork::split, at most kFlatSubs), each on contiguous
  // packs and its own sub-connection of every peer.  Per FIFO step every lane takes its 16-B packs of the input, stores each
  // as two LL lines into every peer's slot (the send), then polls the same lines of every peer's
  // slot here and folds the n inputs in the order of thread block 0's reduction table: acc = x_0,
  // acc = fn(acc, x_i), the table listing ranks n-1 down to 0, i.e. the chain tree's x_{n-1} (+)
  // ... (+) x_0, its own input taken from registers at its position, and stores the result.  A
  // lane reads its input before it writes the output, so in-place calls are safe.  Connections
  // are the flat group's all-pairs connections, peer k on the records of thread block k + 1
  // (transport.cc: flatPeers); 8 peers' lines are polled per wait (VGPR addresses only: see
  // primitives.h ldLines16 on SGPR operands in asm).  No scratch, no flag, no second hop.  Its own kernel: the interpreter
  // kernels keep their register budget.
  __device__ __forceinline__ void runFold(const RankWork& w, int wg, FoldShared* fs) {
    tid = threadIdx.x;
    comm = w.comm;
    timeoutTicks = w.timeoutTicks;
    llFlagMask = w.llFlagMask;
    llCleanMask = w.llCleanMask;
    redArg = 0;
    trace = nullptr;  // set up after the prologue's loads are in flight (below)
    nkBuf = nullptr;
    scG = nullptr;
    rcG = nullptr;
    // every kernel argument the prologue's loads need, in one batch (pinArgs)
    const int np = w.foldPeers;
    const int n = (int)w.sizePerChunk;
    const int split = w.split, base = w.foldPacksPerWg, connSplit = w.connSplit, tbStride = w.tbStride;
    const int mode = w.ringColl;
    const char* const images = w.images;
    DevSendConn* const sendG = w.send;
    DevRecvConn* const recvG = w.recv;
    uint64_t* const epochs = w.epochs;
    const void* const sendbuff = w.sendbuff;
    void* const recvbuff = w.recvbuff;
    pinArgs(np, n, split, base, connSplit, tbStride, mode, images, sendG, recvG, epochs, sendbuff, recvbuff);
    constexpr int E = 8 / TS;
    constexpr int G = 8;  // peers per wait
    const int npkAll = (n + PE - 1) / PE;
    // this workgroup's packs: [p0, p0 + npk), the wg-th of RankWork::split contiguous ranges (the
    // first npkAll % split ranges one pack longer), cut into FIFO steps on its own sub-connection
    // of every peer.  The host's quotient: a 64-bit division here ran ahead of the first load
    const int rem = npkAll - base * split;
    const int p0 = wg * base + min(wg, rem);
    const int npk = base + (wg < rem ? 1 : 0);
    const int nlinesFull = (n + E - 1) / E;
    const __amdgpu_buffer_rsrc_t srs = makeRsrc(sendbuff), drs = makeRsrc(recvbuff);
    const bool vec = aligned16(sendbuff) && aligned16(recvbuff);
    // one round trip: thread block 0's image (the fold order), every peer's send and recv
    // records, the launch epoch, and this lane's first input pack (step 0, q = tid: the pack
    // p0 + tid in every FIFO cut; the ReduceScatter reads the blocks the image names instead),
    // so the input's load does not wait for the image's
    u32x4 pre = {0, 0, 0, 0};
    const bool havePre = mode != kRingReduceScatter && tid < npk;
    {
      // issued first: the lane's later waits (for its image unit or record) then cover it too
      if (havePre) pre = loadPack(srs, vec, p0 + tid, n);
      const u32x4* gimg = (const u32x4*)images;
      const int nU = tbStride >> 4;
      for (int i = tid; i < nU; i += kNT) sh->img[i] = gimg[i];
      if (tid >= 64 && tid < 64 + 4 * np) {
        const int k = (tid - 64) >> 2, j = (tid - 64) & 3;
        ((u32x4*)&fs->foldSend[k])[j] = ((const u32x4*)(sendG + (size_t)(k + 1) * connSplit + wg))[j];
      }
      if (tid >= 192 && tid < 192 + 4 * np) {
        const int k = (tid - 192) >> 2, j = (tid - 192) & 3;
        ((u32x4*)&fs->foldRecv[k])[j] = ((const u32x4*)(recvG + (size_t)(k + 1) * connSplit + wg))[j];
      }
      if (tid == 128) {
        sh->aborted = 0;
        sh->epoch = atomicLoadAgent(epochs + wg);  // slot wg of the fold's range
      }
    }
    __syncthreads();
    const uint64_t workIndex = uni(sh->epoch);
    // MSCCL_AMD_TRACE: the workgroup's setup, its one pass as one primitive, its end (slot wg);
    // NPKit: the launch's time sync and the pass as one RECV_REDUCE_COPY_SEND (tb 0's buffer).
    // After the prologue: the kernel-argument loads these branches chain would otherwise delay the
    // prologue's loads (0.4-0.7 us per launch, profiles/r04b_lat.txt)
    t0 = w.trace != nullptr || w.npkit != nullptr ? __builtin_amdgcn_s_memrealtime() : 0;
    if (w.trace != nullptr) {
      trace = w.trace + (size_t)wg * w.traceEvents;
      nev = 1;
      maxEv = w.traceEvents;
    }
    if (w.npkit != nullptr && wg == 0) {
      const NpkitLog* lg = w.npkit;
      nkCap = lg->cap;
      nkBuf = lg->events;
      nkHeadG = lg->heads;
      nkHead = uni(*nkHeadG);
      nk(NPKIT_EVENT_TIME_SYNC_CPU, 0, (uint64_t)(npkitTicksToNs(t0, lg->clockKHz) + lg->cpuOffsetNs));
      nk(NPKIT_EVENT_TIME_SYNC_GPU, 0, t0);
    }
    DevTbHeader hd;
    {
      u32x4 raw = sh->img[0];
      raw = (u32x4){uni(raw.x), uni(raw.y), uni(raw.z), uni(raw.w)};
      __builtin_memcpy(&hd, &raw, sizeof(hd));
    }
    // the collective (RankWork::ringColl): 0 the AllReduce (the flat tree), kRingReduceScatter,
    // kRingAllGather; the image's transfers 0 / 1 carry the AllReduce / ReduceScatter fold orders
    // and transfer 2 the rank of every peer record (then this rank) (transport.cc: ringUpload)
    const DevTransfer* tr0 = (const DevTransfer*)&sh->img[1];
    const int16_t* reds = (const int16_t*)(tr0 + hd.nsteps) + 2 * hd.ndeps;
    const DevTransfer t = loadTransfer(tr0 + (mode == kRingReduceScatter ? 1 : 0));
    const int16_t* order = reds + t.redPtr;
    const int16_t* rankOf = reds + loadTransfer(tr0 + 2).redPtr;
    const int nfold = t.numReds;
    int ownAt = 0, nq = 0;  // peers folded before the own input
    for (int i = 0; i < nfold; i++) {
      const int b = uni((int)order[i]);
      if (b < 0) ownAt = nq;
      else {
        if (tid == 0) fs->perm[nq] = (uint8_t)(b - 1);  // read after the first step's barrier
        nq++;
      }
    }
    // several orders (w.foldChunkPacks = packs per chunk > 0): transfer 3 holds every class's
    // order, transfer 4 every chunk's class (transport.cc: foldImage); a pack folds in its chunk's
    // order (read after the first step's barrier, like perm)
    const int cpk = w.foldChunkPacks;
    if (cpk > 0) {
      const DevTransfer t3 = loadTransfer(tr0 + 3), t4 = loadTransfer(tr0 + 4);
      const int16_t* co = reds + t3.redPtr;
      for (int i = tid; i < t3.srcoff; i += kNT) {  // one lane per class
        int q = 0;
        for (int j = 0; j < nfold; j++) {
          const int b = co[i * nfold + j];
          if (b < 0) fs->cown[i] = (uint8_t)q;
          else fs->cperm[i][q++] = (uint8_t)(b - 1);
        }
      }
      const int16_t* cc = reds + t4.redPtr;
      for (int i = tid; i < t4.srcoff; i += kNT) fs->chunkClass[i] = (uint8_t)cc[i];
    }
    const int slotLines = uni(fs->foldRecv[0].llSlotLines);
    const int slotPacks = slotLines / 2;
    ev(kEvSetup, 0, 0);
    ev(kEvPrimBegin, 0, ((uint32_t)tRRCS << 24) | (uint32_t)min(npk * PE, 0xFFFFFF));
    nk(NPKIT_EVENT_RECV_REDUCE_COPY_SEND_ENTRY, (uint64_t)n * TS);
    int s0 = 0;
    do {
      const int s1 = npk - s0 < slotPacks ? npk : s0 + slotPacks;
      if (tid < np) {
        // lane k: peer k's send credit (llOp's waitSendCredit) and both slots of this step
        DevSendConn& c = fs->foldSend[tid];
        const uint64_t st = c.step;
        if (c.headSeen + kLLFifoSlots < st + 1) {
          Spin spins;
          uint64_t h;
          while ((h = atomicLoadSys(c.head)) + kLLFifoSlots < st + 1)
            if (spinAbort(spins)) break;
          c.headSeen = h;
        }
        fs->fold[tid].out = c.ll + (st % kLLFifoSlots) * (uint64_t)c.llSlotLines;
        fs->fold[tid].sflag = (uint32_t)(st + 1) & llFlagMask;
        const DevRecvConn& r = fs->foldRecv[tid];
        fs->fold[tid].in = r.ll + (r.step % kLLFifoSlots) * (uint64_t)slotLines;
        fs->fold[tid].rflag = (uint32_t)(r.step + 1) & llFlagMask;
      }
      __syncthreads();
      for (int q = tid; q < s1 - s0; q += kNT) {
        const int B = p0 + s0 + q;
        const bool two = 2 * B + 1 < nlinesFull;
        const uint32_t o0 = (uint32_t)llLineIdx(q, 0) * 16;
        const uint32_t o1 = two ? (uint32_t)llLineIdx(q, 1) * 16 : o0;
        u32x4 own;
        if (mode == kRingReduceScatter) {
          // the send: block rank(k) of the input to peer k, 8 peers' packs loaded per batch
          for (int g0 = 0; g0 < np; g0 += G) {
            u32x4 v[G];
#pragma unroll
            for (int k = 0; k < G; k++)
              if (g0 + k < np) v[k] = loadBlockPack((const T*)w.sendbuff, uni((int)rankOf[g0 + k]), n, B);
#pragma unroll
            for (int k = 0; k < G; k++) {
              if (g0 + k >= np) continue;
              const __amdgpu_buffer_rsrc_t frs = makeRsrc(fs->fold[g0 + k].out);
              const uint32_t f = fs->fold[g0 + k].sflag;
              st16<kAuxFifo>(frs, o0, (u32x4){v[k].x, f, v[k].y, f});
              if (two) st16<kAuxFifo>(frs, o1, (u32x4){v[k].z, f, v[k].w, f});
            }
          }
          own = loadBlockPack((const T*)w.sendbuff, uni((int)rankOf[np]), n, B);
        } else {
          own = s0 == 0 && q == tid && havePre ? pre : loadPack(srs, vec, B, n);
          for (int k = 0; k < np; k++) {  // the send: this pack to every peer
            const __amdgpu_buffer_rsrc_t frs = makeRsrc(fs->fold[k].out);
            const uint32_t f = fs->fold[k].sflag;
            st16<kAuxFifo>(frs, o0, (u32x4){own.x, f, own.y, f});
            if (two) st16<kAuxFifo>(frs, o1, (u32x4){own.z, f, own.w, f});
          }
        }
        if (mode == kRingAllGather) {
          // every peer's pack to its block of the output, peers in record order, 8 per wait
          for (int g0 = 0; g0 < np; g0 += G) {
            const void* la[2 * G];
#pragma unroll
            for (int k = 0; k < G; k++) {
              const char* in = (const char*)fs->fold[g0 + k < np ? g0 + k : g0].in;
              la[2 * k] = in + o0;
              la[2 * k + 1] = in + o1;
            }
            u32x4 ln[2 * G];
            ldLinesPeers<G>(la, ln);
#pragma unroll
            for (int k = 0; k < G; k++) {
              if (g0 + k >= np) continue;
              const uint32_t rflag = fs->fold[g0 + k].rflag;
              Spin spins;
              while (ln[2 * k].y != rflag || ln[2 * k].w != rflag || ln[2 * k + 1].y != rflag ||
                     ln[2 * k + 1].w != rflag) {
                if (spinAbort(spins)) break;
                ldLines2(la[2 * k], la[2 * k + 1], ln[2 * k], ln[2 * k + 1]);
              }
              storeBlockPack((T*)w.recvbuff, uni((int)rankOf[g0 + k]), n, B,
                             (u32x4){ln[2 * k].x, ln[2 * k].z, ln[2 * k + 1].x, ln[2 * k + 1].z});
            }
          }
          storeBlockPack((T*)w.recvbuff, uni((int)rankOf[np]), n, B, own);
          continue;
        }
        u32x4 acc = (u32x4){0, 0, 0, 0};
        bool first = true;
        // this pack's fold order: the schedule's one, or its chunk's class's (per lane)
        const uint8_t* pm = fs->perm;
        int ownPos = ownAt;
        if (cpk > 0) {
          const int cls = fs->chunkClass[B / cpk];
          pm = fs->cperm[cls];
          ownPos = fs->cown[cls];
        }
        for (int g0 = 0; g0 < nq; g0 += G) {  // the fold, peers in fold order
          const void* la[2 * G];
          int pk[G];
#pragma unroll
          for (int k = 0; k < G; k++) {
            pk[k] = pm[g0 + k < nq ? g0 + k : g0];
            const char* in = (const char*)fs->fold[pk[k]].in;
            la[2 * k] = in + o0;
            la[2 * k + 1] = in + o1;
          }
          u32x4 ln[2 * G];
          ldLinesPeers<G>(la, ln);
#pragma unroll
          for (int k = 0; k < G; k++) {
            const int p = g0 + k;
            if (p >= nq) continue;
            if (p == ownPos) {
              acc = first ? own : F::pack(acc, own);
              first = false;
            }
            const uint32_t rflag = fs->fold[pk[k]].rflag;
            Spin spins;
            while (ln[2 * k].y != rflag || ln[2 * k].w != rflag || ln[2 * k + 1].y != rflag ||
                   ln[2 * k + 1].w != rflag) {
              if (spinAbort(spins)) break;
              ldLines2(la[2 * k], la[2 * k + 1], ln[2 * k], ln[2 * k + 1]);
            }
            const u32x4 peer = {ln[2 * k].x, ln[2 * k].z, ln[2 * k + 1].x, ln[2 * k + 1].z};
            acc = first ? peer : F::pack(acc, peer);
            first = false;
          }
        }
        if (ownPos == nq) acc = first ? own : F::pack(acc, own);
        storePack(drs, vec, B, n, acc);
      }
      for (int k = 0; k < np; k++) {
        // LL cleanup (prims_ll.h:90-97): on cleanup steps stamp the send slot's unused lines
        const uint64_t st = uni(fs->foldSend[k].step);
        if ((st & llCleanMask) != llCleanMask) continue;
        const __amdgpu_buffer_rsrc_t frs = makeRsrc(fs->fold[k].out);
        const uint32_t f = fs->fold[k].sflag;
        for (int l = tid; l < slotLines; l += kNT) {
          const int q = ((l >> 7) << 6) + (l & 63), h = (l >> 6) & 1;
          const bool used = s0 + q < s1 && 2 * (p0 + s0 + q) + h < nlinesFull;
          if (!used) st16<kAuxFifo>(frs, (uint32_t)l * 16, (u32x4){0, f, 0, f});
        }
      }
      __syncthreads();
      if (tid < np) {  // this step's slots are consumed / filled: free the peer's slot (head post)
        fs->foldSend[tid].step++;
        const uint64_t rs = fs->foldRecv[tid].step + 1;
        fs->foldRecv[tid].step = rs;
        atomicStoreSys(fs->foldRecv[tid].remoteHead, rs);
      }
      s0 = s1;
    } while (s0 < npk);
    nk(NPKIT_EVENT_RECV_REDUCE_COPY_SEND_EXIT, (uint64_t)n * TS);
    ev(kEvPrimEnd, 0, 0);
    __syncthreads();
    if (tid < np) {  // persist the connections' steps (flat records of thread block k + 1)
      DevSendConn* cg = w.send + (size_t)(tid + 1) * w.connSplit + wg;
      cg->step = fs->foldSend[tid].step;
      cg->headSeen = fs->foldSend[tid].headSeen;
      (w.recv + (size_t)(tid + 1) * w.connSplit + wg)->step = fs->foldRecv[tid].step;
    }
    // the epochs: the fold's workgroups own slots [0, split) of its range (kFlatSubs slots); slots
    // [split, epochSlots) are advanced for the workgroups this call does not run
    __syncthreads();
    const int wgs = w.split;
    if (tid == 0) atomicStoreAgent(w.epochs + wg, workIndex + 1);
    for (int j = wgs + wg + tid * wgs; j < w.epochSlots; j += kNT * wgs) atomicStoreAgent(w.epochs + j, workIndex + 1);
    if (nkBuf != nullptr && tid == 0) *nkHeadG = nkHead;
    ev(kEvEnd, 0, 0);
    if (trace != nullptr && tid == 0) {
      TraceEvent h;
      h.ts = t0;
      h.type = kEvHeader;
      h.step = (uint16_t)nev;
      h.arg = (uint32_t)workIndex;
      trace[0] = h;
    }
  }

  // ---------------------------------------------------------------- the two-phase fold
  // A lowered schedule's large call (lower.h: FoldLowering::twoPhase; plan.cc: lowerToFoldPlan;
  // the msccl-tools two-phase all-pairs, RCCL's allreduce-allpairs files): the schedule's values
  // without its scratch.  The schedule moves chunk c of every rank's input into owner[c]'s scratch
  // (`s`, `r`), the owner folds the n copies with `re` (acc = own, acc = fn(acc, s_i) in its
  // reduction order, prims_ll.h:347-362) and sends the result to every peer (`s`, `r`), i.e. per
  // element 7.5 S (2 ranks) / 11.6 S (8 ranks) HBM bytes per rank.  Here the owner folds straight
  // from the FIFO lines, in the same order, and sends the result on in the same pass: 6 S / 9 S.
  //
  // Every rank owns K chunks of Q packs (transfer 5 of the image lists them per peer record, then
  // this rank's); owned pack m of rank q is pack m % Q of its chunk m / Q (lists[q][m / Q]).  All
  // ranks deal m over their workgroups the same way (RankWork::foldPacksPerWg): workgroup wg owns
  // m in [p0, p0 + npk) of every rank's set and talks to workgroup wg of every peer over flat
  // sub-connection wg.  Per FIFO step (slotPacks of those m), every peer connection carries two
  // slots: (A) this rank's packs of the peer's set, (B) the owner's results.  For every step j a
  // workgroup
  //   A(j): sends its input's packs of every peer's set to that peer (slot A);
  //   B(j): polls every peer's slot-A lines of its own set, folds them with its own input in its
  //      chunk's class order (the order lower.cc read off the schedule), stores the result and
  //      sends it to every peer (slot B);
  //   C(j): polls every peer's slot-B lines and stores each owner's result in its place.
  // A lane reads an input pack (A, B) before it writes that pack (B, C), and the steps in flight
  // at once own disjoint packs: in-place calls are safe.  The three phases are software-pipelined
  // over the steps (below); no workgroup waits on a peer's step the peer has not reached, so the
  // loop cannot deadlock.
#ifndef MSCCL_TP_OCC
#define MSCCL_TP_OCC 1
#endif
  static __device__ __forceinline__ uint32_t divQ(uint32_t m, uint32_t magic, int sh1, int sh2) {
    const uint32_t t = __umulhi(m, magic);
    return (t + ((m - t) >> sh1)) >> sh2;
  }
  __device__ __forceinline__ void runTwoPhase(const RankWork& w, int wg, FoldShared* fs) {
    tid = threadIdx.x;
    comm = w.comm;
    timeoutTicks = w.timeoutTicks;
    llFlagMask = w.llFlagMask;
    llCleanMask = w.llCleanMask;
    redArg = 0;
    trace = nullptr;
    nkBuf = nullptr;
    scG = nullptr;
    rcG = nullptr;
    const int np = w.foldPeers;
    const int n = (int)w.sizePerChunk;  // elements of the whole buffer
    const int wgs = w.split, base = w.foldPacksPerWg, connSplit = w.connSplit, tbStride = w.tbStride;
    const int M = (int)w.tpOwnedPacks, Q = w.foldChunkPacks;
    const uint32_t magic = w.tpMagic;
    const int sh1 = w.tpSh1, sh2 = w.tpSh2;
    const char* const images = w.images;
    DevSendConn* const sendG = w.send;
    DevRecvConn* const recvG = w.recv;
    uint64_t* const epochs = w.epochs;
    const void* const sendbuff = w.sendbuff;
    void* const recvbuff = w.recvbuff;
    pinArgs(np, n, wgs, base, connSplit, tbStride, images, sendG, recvG, epochs, sendbuff, recvbuff);
    // peers per wait / per batch of loads: 8, or 4 in the build for two workgroups per CU
    // (MSCCL_TP_OCC = 2, a measurement variant: <= 128 VGPRs)
    constexpr int G = MSCCL_TP_OCC == 1 ? 8 : 4;
    const int rem = M - base * wgs;
    const int p0 = wg * base + min(wg, rem);
    const int npk = base + (wg < rem ? 1 : 0);
    const __amdgpu_buffer_rsrc_t srs = makeRsrc(sendbuff), drs = makeRsrc(recvbuff);
    const bool vec = aligned16(sendbuff) && aligned16(recvbuff);
    {
      // one round trip: the image (orders, classes, owner lists), every peer's records, the epoch
      const u32x4* gimg = (const u32x4*)images;
      const int nU = tbStride >> 4;
      for (int i = tid; i < nU; i += kNT) sh->img[i] = gimg[i];
      if (tid >= 64 && tid < 64 + 4 * np) {
        const int k = (tid - 64) >> 2, j = (tid - 64) & 3;
        ((u32x4*)&fs->foldSend[k])[j] = ((const u32x4*)(sendG + (size_t)(k + 1) * connSplit + wg))[j];
      }
      if (tid >= 192 && tid < 192 + 4 * np) {
        const int k = (tid - 192) >> 2, j = (tid - 192) & 3;
        ((u32x4*)&fs->foldRecv[k])[j] = ((const u32x4*)(recvG + (size_t)(k + 1) * connSplit + wg))[j];
      }
      if (tid == 128) {
        sh->aborted = 0;
        sh->epoch = atomicLoadAgent(epochs + wg);
      }
    }
    __syncthreads();
    const uint64_t workIndex = uni(sh->epoch);
    DevTbHeader hd;
    {
      u32x4 raw = sh->img[0];
      raw = (u32x4){uni(raw.x), uni(raw.y), uni(raw.z), uni(raw.w)};
      __builtin_memcpy(&hd, &raw, sizeof(hd));
    }
    const DevTransfer* tr0 = (const DevTransfer*)&sh->img[1];
    const int16_t* reds = (const int16_t*)(tr0 + hd.nsteps) + 2 * hd.ndeps;
    const int nfold = loadTransfer(tr0).numReds;
    const DevTransfer t3 = loadTransfer(tr0 + 3), t4 = loadTransfer(tr0 + 4), t5 = loadTransfer(tr0 + 5);
    {
      const int16_t* co = reds + t3.redPtr;
      for (int i = tid; i < t3.srcoff; i += kNT) {  // one lane per class: its peer records in fold order
        int q = 0;
        for (int j = 0; j < nfold; j++) {
          const int b = co[i * nfold + j];
          if (b < 0) fs->cown[i] = (uint8_t)q;
          else fs->cperm[i][q++] = (uint8_t)(b - 1);
        }
      }
      const int16_t* cc = reds + t4.redPtr;
      for (int i = tid; i < t4.srcoff; i += kNT) fs->chunkClass[i] = (uint8_t)cc[i];
    }
    const int16_t* lists = reds + t5.redPtr;  // [peer record k (np: this rank)][K] owned chunks
    const int K = t5.srcoff;
    const int slotLines = uni(fs->foldRecv[0].llSlotLines);
    // packs per step: at most a slot's (RankWork::tpStepPacks; smaller steps keep the FIFO lines in
    // flight within the MALL)
    const int slotPacks = min(slotLines / 2, (int)w.tpStepPacks);
    // Software pipeline: iteration i sends A(i), folds B(i - 1) and stores C(i - 2), so each of
    // them needs only what the peers did one iteration earlier (A(i - 1), B(i - 2)): a workgroup
    // waits only for a peer a whole iteration behind.  Slots per connection: A(j) at base + 2j,
    // B(j) at base + 2j + 1.  After iteration i a receiver has consumed A(0 .. i - 1) and
    // B(0 .. i - 2): it frees the consumed prefix of its FIFO.  The sender of A(i) needs the
    // peer's head at 2i - 7 or more: at most three iterations ahead of its slowest peer.
    const int nsteps = (npk + slotPacks - 1) / slotPacks;
    auto nsOf = [&](int j) { return min(slotPacks, npk - j * slotPacks); };
    // this lane's pack q of step j: its chunk index j in every owner's list and position in it
    auto packOf = [&](int j, int q, int& jj, int& pos) __attribute__((always_inline)) {
      const uint32_t m = (uint32_t)(p0 + j * slotPacks + q);
      jj = (int)divQ(m, magic, sh1, sh2);
      pos = (int)m - jj * Q;
    };
    for (int i = 0; i <= nsteps + 1; i++) {
      const bool doA = i < nsteps, doB = i >= 1 && i <= nsteps, doC = i >= 2;
      if (tid < np) {
        // lane k: credit for the highest slot this iteration writes (A(i) at 2i, else B(i - 1) at
        // 2i - 1), and the four slots of the iteration
        DevSendConn& c = fs->foldSend[tid];
        const uint64_t b = c.step;  // base: the connection's step at launch start (advanced at the end)
        const uint64_t top = doA ? b + 2 * i + 1 : doB ? b + 2 * i : 0;
        if (top > 0 && c.headSeen + kLLFifoSlots < top) {
          Spin spins;
          uint64_t h;
          while ((h = atomicLoadSys(c.head)) + kLLFifoSlots < top)
            if (spinAbort(spins)) break;
          c.headSeen = h;
        }
        const uint64_t sa = b + 2 * i, sb = b + 2 * i - 1;  // A(i), B(i - 1)
        fs->fold[tid].out = c.ll + (sa % kLLFifoSlots) * (uint64_t)c.llSlotLines;
        fs->fold[tid].sflag = (uint32_t)(sa + 1) & llFlagMask;
        fs->fold2[tid].out = c.ll + (sb % kLLFifoSlots) * (uint64_t)c.llSlotLines;
        fs->fold2[tid].sflag = (uint32_t)(sb + 1) & llFlagMask;
        const DevRecvConn& r = fs->foldRecv[tid];
        const uint64_t ra = r.step + 2 * i - 2, rb = r.step + 2 * i - 3;  // A(i - 1), B(i - 2)
        fs->fold[tid].in = r.ll + (ra % kLLFifoSlots) * (uint64_t)slotLines;
        fs->fold[tid].rflag = (uint32_t)(ra + 1) & llFlagMask;
        fs->fold2[tid].in = r.ll + (rb % kLLFifoSlots) * (uint64_t)slotLines;
        fs->fold2[tid].rflag = (uint32_t)(rb + 1) & llFlagMask;
      }
      __syncthreads();
      if (doA) {
        // A(i): this rank's packs of every peer's set, 8 peers' loads in flight
        const int ns = nsOf(i);
        for (int q = tid; q < ns; q += kNT) {
          int j, pos;
          packOf(i, q, j, pos);
          const uint32_t o0 = (uint32_t)llLineIdx(q, 0) * 16, o1 = (uint32_t)llLineIdx(q, 1) * 16;
          for (int g0 = 0; g0 < np; g0 += G) {
            u32x4 v[G];
#pragma unroll
            for (int k = 0; k < G; k++)
              if (g0 + k < np) v[k] = loadPack(srs, vec, (int)lists[(g0 + k) * K + j] * Q + pos, n);
#pragma unroll
            for (int k = 0; k < G; k++) {
              if (g0 + k >= np) continue;
              const __amdgpu_buffer_rsrc_t frs = makeRsrc(fs->fold[g0 + k].out);
              const uint32_t f = fs->fold[g0 + k].sflag;
              st16<kAuxFifo>(frs, o0, (u32x4){v[k].x, f, v[k].y, f});
              st16<kAuxFifo>(frs, o1, (u32x4){v[k].z, f, v[k].w, f});
            }
          }
        }
      }
      if (doB) {
        // B(i - 1): fold the own set from every peer's A lines, store, send the result
        const int ns = nsOf(i - 1);
        for (int q = tid; q < ns; q += kNT) {
          int j, pos;
          packOf(i - 1, q, j, pos);
          const uint32_t o0 = (uint32_t)llLineIdx(q, 0) * 16, o1 = (uint32_t)llLineIdx(q, 1) * 16;
          const int c = lists[np * K + j];
          const int B = c * Q + pos;
          const u32x4 own = loadPack(srs, vec, B, n);
          const int cls = fs->chunkClass[c];
          const uint8_t* pm = fs->cperm[cls];
          const int ownPos = fs->cown[cls];
          u32x4 acc = (u32x4){0, 0, 0, 0};
          bool first = true;
          for (int g0 = 0; g0 < np; g0 += G) {
            const void* la[2 * G];
            int pk[G];
#pragma unroll
            for (int k = 0; k < G; k++) {
              pk[k] = pm[g0 + k < np ? g0 + k : g0];
              const char* in = (const char*)fs->fold[pk[k]].in;
              la[2 * k] = in + o0;
              la[2 * k + 1] = in + o1;
            }
            u32x4 ln[2 * G];
            ldLinesPeers<G>(la, ln);
#pragma unroll
            for (int k = 0; k < G; k++) {
              const int p = g0 + k;
              if (p >= np) continue;
              if (p == ownPos) {
                acc = first ? own : F::pack(acc, own);
                first = false;
              }
              const uint32_t rflag = fs->fold[pk[k]].rflag;
              Spin spins;
              while (ln[2 * k].y != rflag || ln[2 * k].w != rflag || ln[2 * k + 1].y != rflag ||
                     ln[2 * k + 1].w != rflag) {
                if (spinAbort(spins)) break;
                ldLines2(la[2 * k], la[2 * k + 1], ln[2 * k], ln[2 * k + 1]);
              }
              const u32x4 peer = {ln[2 * k].x, ln[2 * k].z, ln[2 * k + 1].x, ln[2 * k + 1].z};
              acc = first ? peer : F::pack(acc, peer);
              first = false;
            }
          }
          if (ownPos == np) acc = first ? own : F::pack(acc, own);
          storePack(drs, vec, B, n, acc);
          for (int k = 0; k < np; k++) {
            const __amdgpu_buffer_rsrc_t frs = makeRsrc(fs->fold2[k].out);
            const uint32_t f = fs->fold2[k].sflag;
            st16<kAuxFifo>(frs, o0, (u32x4){acc.x, f, acc.y, f});
            st16<kAuxFifo>(frs, o1, (u32x4){acc.z, f, acc.w, f});
          }
        }
      }
      if (doC) {
        // C(i - 2): every owner's result to its place, 8 peers per wait
        const int ns = nsOf(i - 2);
        for (int q = tid; q < ns; q += kNT) {
          int j, pos;
          packOf(i - 2, q, j, pos);
          const uint32_t o0 = (uint32_t)llLineIdx(q, 0) * 16, o1 = (uint32_t)llLineIdx(q, 1) * 16;
          for (int g0 = 0; g0 < np; g0 += G) {
            const void* la[2 * G];
#pragma unroll
            for (int k = 0; k < G; k++) {
              const char* in = (const char*)fs->fold2[g0 + k < np ? g0 + k : g0].in;
              la[2 * k] = in + o0;
              la[2 * k + 1] = in + o1;
            }
            u32x4 ln[2 * G];
            ldLinesPeers<G>(la, ln);
#pragma unroll
            for (int k = 0; k < G; k++) {
              if (g0 + k >= np) continue;
              const uint32_t rflag = fs->fold2[g0 + k].rflag;
              Spin spins;
              while (ln[2 * k].y != rflag || ln[2 * k].w != rflag || ln[2 * k + 1].y != rflag ||
                     ln[2 * k + 1].w != rflag) {
                if (spinAbort(spins)) break;
                ldLines2(la[2 * k], la[2 * k + 1], ln[2 * k], ln[2 * k + 1]);
              }
              storePack(drs, vec, (int)lists[(g0 + k) * K + j] * Q + pos, n,
                        (u32x4){ln[2 * k].x, ln[2 * k].z, ln[2 * k + 1].x, ln[2 * k + 1].z});
            }
          }
        }
      }
      for (int k = 0; k < np; k++) {
        // LL cleanup (prims_ll.h:90-97): on cleanup steps stamp the unused lines of a slot sent
        const uint64_t b = uni(fs->foldSend[k].step);
        for (int h2 = 0; h2 < 2; h2++) {
          if (h2 == 0 ? !doA : !doB) continue;
          const uint64_t st = h2 == 0 ? b + 2 * i : b + 2 * i - 1;
          if ((st & llCleanMask) != llCleanMask) continue;
          const int ns = nsOf(h2 == 0 ? i : i - 1);
          const FoldShared::Peer& pr = h2 == 0 ? fs->fold[k] : fs->fold2[k];
          const __amdgpu_buffer_rsrc_t frs = makeRsrc(pr.out);
          const uint32_t f = pr.sflag;
          for (int l = tid; l < slotLines; l += kNT) {
            const int q = ((l >> 7) << 6) + (l & 63);
            if (q >= ns) st16<kAuxFifo>(frs, (uint32_t)l * 16, (u32x4){0, f, 0, f});
          }
        }
      }
      __syncthreads();
      if (tid < np && (doB || doC)) {
        // consumed: A(0 .. a - 1), B(0 .. b - 1): free the prefix (head post)
        const int a = min(i, nsteps), b = max(0, min(i - 1, nsteps));
        const uint64_t head = fs->foldRecv[tid].step + (uint64_t)(a > b ? 2 * b + 1 : 2 * a);
        atomicStoreSys(fs->foldRecv[tid].remoteHead, head);
      }
    }
    if (tid < np) {  // both counters advance by the launch's slots
      fs->foldSend[tid].step += 2 * (uint64_t)nsteps;
      fs->foldRecv[tid].step += 2 * (uint64_t)nsteps;
    }
    __syncthreads();
    if (tid < np) {  // persist the connections' steps (flat records of thread block k + 1)
      DevSendConn* cg = sendG + (size_t)(tid + 1) * connSplit + wg;
      cg->step = fs->foldSend[tid].step;
      cg->headSeen = fs->foldSend[tid].headSeen;
      (recvG + (size_t)(tid + 1) * connSplit + wg)->step = fs->foldRecv[tid].step;
    }
    // the epochs: slots [0, wgs) are this launch's workgroups', [wgs, epochSlots) advanced for the rest
    if (tid == 0) atomicStoreAgent(epochs + wg, workIndex + 1);
    for (int j = wgs + wg + tid * wgs; j < w.epochSlots; j += kNT * wgs) atomicStoreAgent(epochs + j, workIndex + 1);
  }

  // ---------------------------------------------------------------- small calls
  // A launch whose every rank's call runs run()'s loop as equal passes: one iteration
  // (sizePerChunk <= chunkSize) or full iterations merged `merge` at a time with nothing left
  // over (enqueue.cc: smallEligible), outside the ring / tree fallback and without tracing.
  // Then every pass has nelem = min(sizePerChunk, chunkSize * merge) and needs no chunk
  // arithmetic, offsets fit 32 bits and split is a power of two, so a workgroup's
  // positions are shifts.  The transfers, their cut into calls (run()'s macT and reach rules, so
  // each end of a connection may run either kernel), the flags (iter = pass) and the primitives
  // are run()'s; what goes is the 64-bit iteration arithmetic and most of the scalar state the
  // big loop keeps live (SGPR spills), a few us per launch.
  template <int SET>
  __device__ __forceinline__ void runSmall(const RankWork& w, int local) {
#ifdef MSCCL_LAT_TRACE
    const uint64_t tStart = __builtin_amdgcn_s_memrealtime();  // the measurement build's time origin
#endif
    redArg = 0;
    trace = nullptr;
    nkBuf = nullptr;
    const int split = w.split;
    const int lg = __builtin_ctz((unsigned)split);
    const int bid = local >> lg, sub = local & (split - 1);
    // the prologue's kernel arguments in the entry batch (the compiler otherwise issues the image
    // pointer's load inside the image lanes' branch, after the first wait): 2 ranks, graph replay,
    // same box, 3 alternating runs (profiles/r05r_pin_ab.txt): 8 KiB 6.57 -> 6.43 us, 1 MiB 7.89 ->
    // 7.76, 4 MiB 13.02 -> 12.80
    pinArgs(w.images, w.tbStride, w.send, w.recv, w.epochs, w.connSplit, w.maxSplit, w.comm);
    DevTbHeader hd;
    const uint64_t workIndex = prologue(w, bid, sub, hd);
#ifndef MSCCL_LAT_TRACE
    // MSCCL_AMD_TRACE=2's start stamp: after the prologue (see run())
    const uint64_t tStart = w.trace != nullptr ? __builtin_amdgcn_s_memrealtime() : 0;
#endif
    const int maxSplit = w.maxSplit;
#ifdef MSCCL_LAT_TRACE
    trace = w.trace ? w.trace + (size_t)(bid * maxSplit + sub) * w.traceEvents : nullptr;
    nev = 1;
    maxEv = w.traceEvents;
    LAT_EV(10);
#endif
    T* const bufs[3] = {(T*)w.sendbuff, (T*)w.recvbuff, (T*)w.scratch};
    // element offsets stay below 2^30 (smallEligible: at most 1 GiB per buffer), so 32 bits
    const int sizePer = (int)w.sizePerChunk;
    const int chunk = (int)w.chunkSize;
    const int nelem = sizePer <= chunk ? sizePer : min(sizePer, chunk * (int)w.merge);
    const bool whole = nelem == sizePer;  // run()'s `nelem == sizePer`
    const int mac = w.maxAllowedCount;
    const int64_t maxOp = w.maxOpElems;
    const uint32_t Qc = ((uint32_t)nelem + PE - 1) / PE;
    const int q0 = (int)((Qc * (uint32_t)sub) >> lg), q1 = (int)((Qc * (uint32_t)(sub + 1)) >> lg);
    // One iteration of the ring fallback (enqueue.cc: smallEligible; sizePerChunk 0, so `whole`):
    // run()'s ring arithmetic at grid 0 in 32 bits: runRing's realChunkSize (all_reduce.h:43-48;
    // reduce_scatter.h / all_gather.h: lastChunkSize once the loop covers the rest), offsets from the
    // program's chunk (AllReduce) or rank (ReduceScatter / AllGather) indices, nelem = min(real,
    // size - offset), one workgroup per channel.  Every transfer has count 1 (maxAllowedCount 1).
    const int ringColl = SET == kSetAll ? (int)w.ringColl : 0;
    int ringReal = 0;
    if (ringColl == kRingAllReduce) {
      const int unit = w.nBlocks * (int)w.ringRanks * (int)w.minChunk;
      ringReal = min(chunk, ((int)w.ringSize + unit - 1) / unit * (int)w.minChunk);
    } else if (ringColl != 0) {
      ringReal = (int)w.ringSize < w.nBlocks * chunk ? (int)w.ringLastChunk : chunk;
    }
    // one pass: grid = offset of the pass, iter = its index; false when a transfer ends the tb
    auto runPass = [&](int grid, int iter) __attribute__((always_inline)) -> bool {
      int step = 0;
      for (int i = 0; i < hd.nsteps; i++) {
        DevTransfer t = loadTransfer(&tr[i]);
        const bool fused = fuseable<true>(t);
        if (t.type == tSendRrc && !fused) t.type = tSend;
        const bool sendCpy = t.type == tSendCpy;
        if (sendCpy) t.type = tCopySend;
        const DevTransfer td = fused || sendCpy ? loadTransfer(&tr[i + 1]) : t;
        if (t.numDeps > 0) {
          waitDeps(t, w.flags, workIndex, iter, sub, maxSplit);
          step += t.numDeps - 1;
        }
        T* srcP = bufs[t.srcbuf < 2 ? t.srcbuf : 2];
        T* dstP = bufs[td.dstbuf < 2 ? td.dstbuf : 2];
        int macT = (t.type != tRe && whole && (int64_t)nelem * t.count <= maxOp) ? t.count : mac;
        if ((int64_t)nelem * TS * macT > (int64_t)0x7fffff00) {  // run()'s descriptor-reach cut
          const int64_t reach = (int64_t)0x7fffff00 / ((int64_t)nelem * TS);
          macT = reach < 1 ? 1 : (int)reach;
        }
        for (int c = 0; c < t.count; c += macT) {
          const int thisCount = macT < t.count - c ? macT : t.count - c;
          Shape s;
          int so = grid + (t.srcoff + c) * sizePer, dso = grid + (td.dstoff + c) * sizePer;
          s.n = nelem * thisCount;
          if (ringColl != 0) {
            int lim;
            if (ringColl == kRingAllReduce) {
              so = ((t.srcoff >= 0 ? t.srcoff : t.dstoff) * w.nBlocks + bid) * ringReal;
              dso = so;
              lim = so;
            } else {
              lim = bid * ringReal;
              so = lim + (t.srcoff >= 0 ? t.srcoff * (int)w.ringSize : 0);
              dso = lim + (t.dstoff >= 0 ? t.dstoff * (int)w.ringSize : 0);
            }
            const int ne = min(ringReal, (int)w.ringSize - lim);
            s.n = ne > 0 ? ne : 0;
          }
          if (split == 1) {
            s.Q = (s.n + PE - 1) / PE;
            s.q0 = 0;
            s.Lq = s.Q;
            s.npk = s.Q;
          } else {
            s.Q = (int)Qc;
            s.q0 = q0;
            s.Lq = q1 - q0;
            s.npk = thisCount * s.Lq;
          }
          if (!exec<true, SET>(t, srcP, dstP, so, dso, grid + c * sizePer, sizePer, s)) return false;
          if (t.type == tRe && c == 0) step += t.numReds - 1;
        }
        if (fused || sendCpy) {
          step++;
          i++;
          t = td;
        }
        if (t.hasDep) publishFlag(w.flags, bid * maxSplit + sub, workIndex, iter, step);
        step++;
      }
      return true;
    };
    // the common small call: one pass without loop state; the exchange kernels keep only the loop
    // (one instance of runPass: less code to fetch per launch)
    if (SET != kSetExchange && whole) {
      runPass(0, 0);
    } else {
      for (int grid = 0, iter = 0; grid < sizePer; grid += nelem, iter++)
        if (!runPass(grid, iter)) break;
    }
    LAT_EV(15);
    epilogue(w, bid, sub, workIndex);
#ifdef MSCCL_LAT_TRACE
    LAT_EV(16);
    if (trace != nullptr && tid == 0) {
      TraceEvent e;
      e.ts = tStart;
      e.type = kEvHeader;
      e.step = (uint16_t)nev;
      e.arg = (uint32_t)workIndex;
      trace[0] = e;
    }
    return;
#endif
    if (w.trace != nullptr && tid == 0) {
      // light trace (MSCCL_AMD_TRACE=2): this workgroup's start, and its end with the XCD it ran on
      // (HW_REG_XCC_ID: the dispatch order only says which blocks share an XCD, not which one)
      uint32_t xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      TraceEvent* tr = w.trace + (size_t)(bid * maxSplit + sub) * w.traceEvents;
      TraceEvent e;
      e.ts = __builtin_amdgcn_s_memrealtime();
      e.type = kEvEnd;
      e.step = 0;
      e.arg = xcc & 0xf;
      tr[1] = e;
      e.ts = tStart;
      e.type = kEvHeader;
      e.step = 2;
      e.arg = (uint32_t)workIndex;
      tr[0] = e;
    }
  }
};

// ---------------------------------------------------------------- the pair kernel
template <typename T, int OP>
struct PairRunner : Interp<T, OP, pLL> {
  using I = Interp<T, OP, pLL>;
  using I::PE;
  using I::U;
  // A pair-form schedule (transport.cc: algoUpload) in one pass (enqueue.cc: launchGroup): thread
  // block b's program is one fused s + rrc of input chunk pairSrc + b * pairStride into chunk
  // pairDst + b * pairStride, no dependency.  Everything runSmall would read from the image comes
  // from the kernel arguments, so one memory round trip brings the connection records, the launch
  // epoch and this lane's source packs of the first FIFO step (llFusedOp's cut), and the exchange
  // starts right after it.  The values, FIFO steps and flags are runSmall's (a peer may run either).
  __device__ __forceinline__ void run(const RankWork& w, int local) {
#ifdef MSCCL_LAT_TRACE
    const uint64_t tStart = __builtin_amdgcn_s_memrealtime();  // the measurement build's time origin
#endif
    I& it = *this;
    it.tid = threadIdx.x;
    it.redArg = 0;
    it.trace = nullptr;
    it.nkBuf = nullptr;
    const int split = w.split;
    const int lg = __builtin_ctz((unsigned)split);
    const int bid = local >> lg, sub = local & (split - 1);
    const int sizePer = (int)w.sizePerChunk;
    const int cslot = bid * w.connSplit + sub;
    DevSendConn* const sendG = w.send;
    DevRecvConn* const recvG = w.recv;
    uint64_t* const epochs = w.epochs;
    const int maxSplit = w.maxSplit;
    const int stride = w.pairStride;
    T* const src = (T*)w.sendbuff + (int64_t)(w.pairSrc + bid * stride) * sizePer;
    T* const dst = (T*)(w.pairDstBuf ? w.recvbuff : w.sendbuff) + (int64_t)(w.pairDst + bid * stride) * sizePer;
    pinArgs(split, sizePer, cslot, sendG, recvG, epochs, maxSplit, src, dst);
    // this workgroup's positions of the chunk (runSmall's cut for one chunk of nelem = sizePer)
    const uint32_t Qc = ((uint32_t)sizePer + PE - 1) / PE;
    Shape s;
    s.n = sizePer;
    s.Q = (int)Qc;
    // (64-bit products: the lowered pair runs one chunk of up to 1 GiB over up to kMaxFlatSubs
    // workgroups; where runSmall's 32-bit cut holds, both cut alike)
    s.q0 = split == 1 ? 0 : (int)(((uint64_t)Qc * (uint32_t)sub) >> lg);
    s.Lq = split == 1 ? (int)Qc : (int)(((uint64_t)Qc * (uint32_t)(sub + 1)) >> lg) - s.q0;
    s.npk = s.Lq;
    // one round trip: this lane's packs q = tid + u * kNT of step 0 (llFusedOp uses those with
    // q < min(npk, slot packs) <= kNT * U), both connection records (wave 7), the epoch (wave 6)
    u32x4 pre[U];
    {
      const __amdgpu_buffer_rsrc_t srs = makeRsrc(src);
      const bool vec = I::aligned16(src);
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int q = it.tid + u * kNT;
        pre[u] = q < s.npk ? it.loadPack(srs, vec, s.bufPack(q), s.n) : (u32x4){0, 0, 0, 0};
      }
      if (it.tid >= 448 && it.tid < 456) {
        const int j = it.tid - 448;
        const u32x4* from = j < 4 ? (const u32x4*)(sendG + cslot) + j : (const u32x4*)(recvG + cslot) + (j - 4);
        u32x4* to = j < 4 ? (u32x4*)&it.sh->sconn + j : (u32x4*)&it.sh->rconn + (j - 4);
        *to = *from;
      }
      if (it.tid == 384) {
        it.sh->aborted = 0;
        it.sh->epoch = atomicLoadAgent(epochs + bid * maxSplit + sub);
      }
    }
    it.comm = w.comm;
    it.timeoutTicks = w.timeoutTicks;
    it.llFlagMask = w.llFlagMask;
    it.llCleanMask = w.llCleanMask;
    it.refNthreads = w.refNthreads;
    __syncthreads();
    const uint64_t workIndex = uni(it.sh->epoch);
    it.scG = sendG + cslot;
    it.rcG = recvG + cslot;
    it.sc = &it.sh->sconn;
    it.rc = &it.sh->rconn;
    it.sendStep = uni(it.sh->sconn.step);
    it.recvStep = uni(it.sh->rconn.step);
    it.headSeen = uni(it.sh->sconn.headSeen);
    it.tailSeen = uni(it.sh->rconn.tailSeen);
#ifdef MSCCL_LAT_TRACE
    // (tools/lat_trace.py: the same points as runSmall's, in this workgroup's trace slot)
    it.trace = w.trace ? w.trace + (size_t)(bid * maxSplit + sub) * w.traceEvents : nullptr;
    it.nev = 1;
    it.maxEv = w.traceEvents;
    it.ev(10, 0, 0);
#endif
    [[clang::always_inline]] it.template llFusedOp<true, true>(src, dst, s, pre);
#ifdef MSCCL_LAT_TRACE
    it.ev(15, 0, 0);
#endif
    it.epilogue(w, bid, sub, workIndex);
#ifdef MSCCL_LAT_TRACE
    it.ev(16, 0, 0);
    if (it.trace != nullptr && it.tid == 0) {
      TraceEvent e;
      e.ts = tStart;
      e.type = kEvHeader;
      e.step = (uint16_t)it.nev;
      e.arg = (uint32_t)workIndex;
      it.trace[0] = e;
    }
#endif
  }
};

// The rank of the launch that owns block b: ranks' blocks are consecutive ([blockBase, blockBase +
// nBlocks) in rank order), so r = the number of ranks i >= 1 whose blocks start at or below b.  All
// R block bases are independent kernel-argument loads issued together (a search loop over them
// was one dependent scalar load per rank before the prologue could start).
template <int R>
__device__ __forceinline__ int rankOfBlock(const LaunchArgsN<R>& args, int b) {
  int r = 0;
#pragma unroll
  for (int i = 1; i < R; i++) r += (i < args.nRanks && b >= args.w[i].blockBase) ? 1 : 0;
  return r;
}

// Kernel arguments into the scalar cache in one round trip: one load per 64-B line of [p, p +
// BYTES), all issued before the first is used (pinArgs).  The kernel-argument fields a prologue
// reads are spread over a RankWork's four lines, and the compiler issues them in several batches,
// each waiting for the last: every batch that touched a new line paid a cache miss.
template <int BYTES>
__device__ __forceinline__ void warmArgLines(const void* p) {
  const char* c = (const char*)p;
  uint32_t v[(BYTES + 63) / 64];
#pragma unroll
  for (int i = 0; i < (BYTES + 63) / 64; i++) v[i] = *(const uint32_t*)(c + (i * 64 < BYTES - 4 ? i * 64 : BYTES - 4));
#pragma unroll
  for (int i = 0; i < (BYTES + 63) / 64; i++) pinArg(v[i]);
}

// The RankWork of block b, its lines warmed after the lookup in the launches of more than
// kCompactLaunchRanks ranks (8 ranks: 0.2-0.35 us less per launch).  The compact launches do
// without: warming their whole 424-B block first cost 0.2-0.5 us (profiles/r04f_lat.txt).
template <int R>
__device__ __forceinline__ const RankWork& rankWorkOf(const LaunchArgsN<R>& args, int b) {
  const RankWork& w = args.w[rankOfBlock(args, b)];
  if constexpr (R > kCompactLaunchRanks) warmArgLines<sizeof(RankWork)>(&w);
  return w;
}

template <typename T, int OP, int PROTO>
__global__ void __launch_bounds__(kNT, 4) mscclKernel(const LaunchArgs args) {
  __shared__ BlockShared sh;
  const int b = blockIdx.x;
  const RankWork& w = rankWorkOf(args, b);
  const int local = b - w.blockBase;
  Interp<T, OP, PROTO> it;
  it.sh = &sh;
  it.run(w, local / w.split, local % w.split);
}

// Small-call variant (Interp::runSmall): every RankWork of the launch is one interpreter
// iteration of an MSCCL schedule.  SET: the transfer types its programs use (devcomm.h).
template <typename T, int OP, int PROTO, int R, int SET>
__global__ void __launch_bounds__(kNT, 4) mscclSmallKernel(const LaunchArgsN<R> args) {
  __shared__ BlockShared sh;
  const int b = blockIdx.x;
  const RankWork& w = rankWorkOf(args, b);
  Interp<T, OP, PROTO> it;
  it.sh = &sh;
  it.template runSmall<SET>(w, b - w.blockBase);
}

// The pair kernel (PairRunner): every RankWork of the launch is a pair-form schedule in one pass.
template <typename T, int OP, int R>
__global__ void __launch_bounds__(kNT, 4) mscclPairKernel(const LaunchArgsN<R> args) {
  __shared__ BlockShared sh;
  const int b = blockIdx.x;
  const RankWork& w = rankWorkOf(args, b);
  PairRunner<T, OP> it;
  it.sh = &sh;
  it.run(w, b - w.blockBase);
}

// The flat tree's fold kernel (Interp::runFold): rank r of the launch owns workgroups
// [blockBase, blockBase + nBlocks).
template <typename T, int OP, int R>
__global__ void __launch_bounds__(kNT, 1) mscclFoldKernel(const LaunchArgsN<R> args) {
  __shared__ BlockShared sh;
  __shared__ FoldShared fs;
  const int b = blockIdx.x;
  const RankWork& w = rankWorkOf(args, b);
  Interp<T, OP, pLL> it;
  it.sh = &sh;
  it.runFold(w, b - w.blockBase, &fs);
}

// The two-phase fold (Interp::runTwoPhase): rank r of the launch owns workgroups [blockBase,
// blockBase + nBlocks), one per flat sub-connection.
// MSCCL_TP_OCC: workgroups per CU the kernel is built for (1; 2: four waves per SIMD, <= 128
// VGPRs, 4 peers per batch of loads; a measurement variant)
template <typename T, int OP, int R>
__global__ void __launch_bounds__(kNT, MSCCL_TP_OCC == 1 ? 1 : 4) mscclTwoPhaseKernel(const LaunchArgsN<R> args) {
  __shared__ BlockShared sh;
  __shared__ FoldShared fs;
  const int b = blockIdx.x;
  const RankWork& w = rankWorkOf(args, b);
  Interp<T, OP, pLL> it;
  it.sh = &sh;
  it.runTwoPhase(w, b - w.blockBase, &fs);
}


// ---------------------------------------------------------------- the direct form (Simple)
// A Simple schedule's call when every rank of the communicator is in this launch (lower.h:
// DirectLowering; enqueue.cc: launchGroup).  The reference's P2P direct mode lets a sender write
// straight into the receiver's buffer inside one process (prims_simple.h:75-128, 500-560, the
// pointer travelling through ptrExchange, comm.h:39); within one fused launch every rank's buffers
// are addressable and ready when it starts, so no FIFO, flag or pointer exchange is needed: the
// launch's argument block holds every rank's RankWork, in rank order.  Rank r's workgroups
//   AllGather:     copy r's input to block r of every rank's output (read once, written n times);
//   ReduceScatter: fold block r of every rank's input in the schedule's order of the pack's
//                  chunk class and store r's output;
//   AllReduce:     fold their share of every rank's input (the same order on every rank) and
//                  store the result into every rank's output.
// A lane reads every operand of a pack before it writes that pack anywhere, and no other lane
// of the launch reads or writes it: in-place AllReduce calls are safe.
#ifndef MSCCL_DIRECT_UD
#define MSCCL_DIRECT_UD 4
#endif
struct alignas(16) DirectShared {
  const void* rankBuf[kMaxLaunchRanks];                // every rank's input, by rank
  uint8_t perm[kMaxDirectClasses][kMaxLaunchRanks];    // per class: the ranks in fold order
  uint8_t chunkClass[kMaxFoldChunks];                  // per output chunk: its class
};

template <typename T, int OP>
struct DirectRunner : Interp<T, OP, pSimple> {
  using I = Interp<T, OP, pSimple>;
  using I::PE;
  using F = typename I::F;
  static constexpr int UD = MSCCL_DIRECT_UD;  // packs per lane per pass (n loads each in flight)
  // pack B of a block of n elements at a per-lane address (the rank whose operand a lane loads
  // follows its pack's chunk class, so a wave's lanes may read different ranks' buffers: no
  // wave-uniform buffer descriptor)
  static __device__ __forceinline__ u32x4 ldPackLane(const T* base, int B, int n) {
    const int e0 = B * PE;
    const int ne = n - e0;
    if (ne >= PE && (((uintptr_t)base & 15) == 0)) return *(const u32x4*)(base + e0);
    T v[PE];
#pragma unroll
    for (int i = 0; i < PE; i++) {
      if (i < ne) v[i] = base[e0 + i];
      else __builtin_memset(&v[i], 0, sizeof(T));
    }
    u32x4 o;
    __builtin_memcpy(&o, v, 16);
    return o;
  }
  template <int R>
  __device__ __forceinline__ void run(const LaunchArgsN<R>& args, const RankWork& w, int wg, DirectShared* fs) {
    I& it = *this;
    it.tid = threadIdx.x;
    const int tid = it.tid;
    const int n = args.nRanks;
    const int me = w.directRank;
    const int mode = w.ringColl;
    const int64_t count = w.sizePerChunk;  // elements of one rank block (AG: input, RS: output, AR: buffer)
    const int wgs = w.split;
    const int Q = w.foldChunkPacks;        // packs per chunk (RS / AR), for the chunk's class
    const uint32_t magic = w.tpMagic;
    const int sh1 = w.tpSh1, sh2 = w.tpSh2;
    // the fold orders of this rank (image: transfer 0 the orders, ranks per class; transfer 1 the
    // class of every chunk), read from the image in global memory into LDS
    if (mode != kRingAllGather) {
      const char* img = (const char*)w.images;
      const DevTbHeader* hd = (const DevTbHeader*)img;
      const DevTransfer* tr0 = (const DevTransfer*)(img + sizeof(DevTbHeader));
      const int16_t* reds = (const int16_t*)(tr0 + hd->nsteps) + 2 * hd->ndeps;
      const int nOrd = tr0[0].srcoff * n, p0r = tr0[0].redPtr, nCh = tr0[1].srcoff, p1r = tr0[1].redPtr;
      for (int i = tid; i < nOrd; i += kNT) fs->perm[i / n][i % n] = (uint8_t)reds[p0r + i];
      for (int i = tid; i < nCh; i += kNT) fs->chunkClass[i] = (uint8_t)reds[p1r + i];
    }
    for (int q = 0; q < n; q++)  // (a uniform index: kernel-argument loads stay scalar)
      if (tid == q) fs->rankBuf[q] = args.w[q].sendbuff;  // the per-lane rank choice below reads LDS
    __syncthreads();
    const int64_t npkAll = (count + PE - 1) / PE;
    // this workgroup's packs: AG / RS the whole rank block, AR this rank's share of it
    int64_t lo = 0, hi = npkAll;
    if (mode == kRingAllReduce) {
      lo = npkAll * me / n;
      hi = npkAll * (me + 1) / n;
    }
    const int64_t span = hi - lo;
    const int64_t p0 = lo + span * wg / wgs, p1 = lo + span * (wg + 1) / wgs;
    const int64_t rsOff = mode == kRingReduceScatter ? (int64_t)me * count : 0;  // RS: block me of every input
    for (int64_t base = p0; base < p1; base += (int64_t)kNT * UD) {
      int B[UD];
      bool act[UD];
#pragma unroll
      for (int u = 0; u < UD; u++) {
        const int64_t b = base + tid + (int64_t)u * kNT;
        act[u] = b < p1;
        B[u] = act[u] ? (int)b : 0;
      }
      if (mode == kRingAllGather) {
        const T* src = (const T*)args.w[me].sendbuff;
        const __amdgpu_buffer_rsrc_t srs = makeRsrc(src);
        const bool sv = I::aligned16(src);
        u32x4 v[UD];
#pragma unroll
        for (int u = 0; u < UD; u++) v[u] = act[u] ? it.loadPack(srs, sv, B[u], (int)count) : (u32x4){0, 0, 0, 0};
        for (int q = 0; q < n; q++) {
          T* dst = (T*)args.w[q].recvbuff + (int64_t)me * count;
          const __amdgpu_buffer_rsrc_t drs = makeRsrc(dst);
          const bool dv = I::aligned16(dst);
#pragma unroll
          for (int u = 0; u < UD; u++)
            if (act[u]) it.storePack(drs, dv, B[u], (int)count, v[u]);
        }
        continue;
      }
      // RS / AR: every rank's pack, folded in the order of the pack's chunk class
      u32x4 acc[UD];
      const uint8_t* pm[UD];
#pragma unroll
      for (int u = 0; u < UD; u++) {
        const uint32_t c = Q > 0 ? (uint32_t)I::divQ((uint32_t)B[u], magic, sh1, sh2) : 0;
        pm[u] = fs->perm[fs->chunkClass[c]];
      }
      for (int j = 0; j < n; j++) {
        u32x4 v[UD];
#pragma unroll
        for (int u = 0; u < UD; u++) {
          const int q = pm[u][j];
          v[u] = act[u] ? ldPackLane((const T*)fs->rankBuf[q] + rsOff, B[u], (int)count) : (u32x4){0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < UD; u++) acc[u] = j == 0 ? v[u] : F::pack(acc[u], v[u]);
      }
      const int nOut = mode == kRingAllReduce ? n : 1;
      for (int q0 = 0; q0 < nOut; q0++) {
        const int q = mode == kRingAllReduce ? q0 : me;
        T* dst = (T*)args.w[q].recvbuff;
        const __amdgpu_buffer_rsrc_t drs = makeRsrc(dst);
        const bool dv = I::aligned16(dst);
#pragma unroll
        for (int u = 0; u < UD; u++)
          if (act[u]) it.storePack(drs, dv, B[u], (int)count, acc[u]);
      }
    }
  }
};

// The direct form (DirectRunner): every rank of the communicator in this launch, RankWork in rank
// order; rank r owns workgroups [blockBase, blockBase + nBlocks).
template <typename T, int OP, int R>
__global__ void __launch_bounds__(kNT, 2) mscclDirectKernel(const LaunchArgsN<R> args) {
  __shared__ DirectShared ds;
  const int b = blockIdx.x;
  const RankWork& w = rankWorkOf(args, b);
  DirectRunner<T, OP> it;
  it.sh = nullptr;  // no program image in LDS
  it.run(args, w, b - w.blockBase, &ds);
}

}  // namespace msccl

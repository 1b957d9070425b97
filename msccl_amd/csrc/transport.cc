// xGMI peer transport for MSCCL connections.
//
// Replaces the reference's P2P transport (transport/p2p.cc:143-344) and the MSCCL connect block
// of initTransportsRank (init.cc:781-874):
//   * one connection per (channel, peer) and direction, as named by the XML thread blocks.  The
//     reference shares a (channel, peer) connection between all loaded algorithms; here every
//     algorithm (and the ring fallback) owns its connections, so a connection belongs to exactly
//     one (algorithm, thread block, sub-workgroup) and its persistent step counters sit at an
//     address the kernel computes from its block index alone (no dependent load in the kernel
//     prologue).  The FIFO memory this costs is small next to 288 GB of HBM;
//   * the receiver owns the FIFOs (LL: 8 steps x 4096 16-B lines; Simple: 8 x 512 KiB by default,
//     NCCL_LL_BUFFSIZE / NCCL_BUFFSIZE override) and a tail word; the sender owns a head word the
//     receiver writes.  All of it lives in one uncached (fine-grained) HBM arena per rank,
//     exported once per rank (hipIpc) or shared by pointer inside a process;
//   * a rank's layout is published as a table [group][channel][peer] -> offsets and exchanged.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <map>

#include "comm.h"
#include "debug.h"

namespace msccl {

namespace {
constexpr size_t kWordStride = 128;   // head/tail words on their own 128-B lines
constexpr size_t kFifoAlign = 4096;
size_t alignUp(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Protocols whose FIFO memory a group needs (LL and LL128 share the LL FIFO).
uint8_t groupProtoMask(const ncclComm* comm, int group) {
  if (group == kRingGroup || group == kTreeGroup) return (uint8_t)((1u << kProtoLL) | (1u << kProtoSimple));
  if (group == kFlatGroup) return (uint8_t)(1u << kProtoLL);
  uint8_t m = (uint8_t)(1u << comm->algos[group].proto);
  for (auto& r : comm->regs)
    if (r.algoIndex == group) m |= (uint8_t)(1u << r.proto);
  if (m & (1u << kProtoLL128)) m |= (uint8_t)(1u << kProtoLL);  // LL128 may run as LL (remote peers)
  return m;
}

int groupSubs(const ncclComm* comm, int group) {
  if (group == kFlatGroup) return comm->flatSubs;  // one per fold / pair / two-phase workgroup
  if (group == kRingGroup || group == kTreeGroup) return 1;  // the ring / tree fallbacks run unsplit
  return comm->algoSplit.empty() ? 1 : comm->algoSplit[group];
}
// The tree fallback's chain (rank order, root 0): thread block 2c+0 reduces up (receives from
// the child, sends to the parent; the root sends its result back down to the child), 2c+1
// broadcasts down (receives from the parent, sends to the child; empty on the root).
void treePeers(int rank, int n, std::vector<int>* sp, std::vector<int>* rp) {
  const int parent = rank - 1, child = rank + 1 < n ? rank + 1 : -1;
  sp->assign(2 * kRingChannels, -1);
  rp->assign(2 * kRingChannels, -1);
  for (int c = 0; c < kRingChannels; c++) {
    if (rank == 0) {
      (*rp)[2 * c] = child;
      (*sp)[2 * c] = child;
    } else {
      (*rp)[2 * c] = child;
      (*sp)[2 * c] = parent;
      (*rp)[2 * c + 1] = parent;
      (*sp)[2 * c + 1] = child;
    }
  }
}
// The flat tree's thread blocks: 0 folds (no peer), 1 + j exchanges with the j-th peer in
// ascending rank order (sends to it and receives from it, channel 0).
void flatPeers(int rank, int n, std::vector<int>* sp, std::vector<int>* rp) {
  sp->assign(n, -1);
  rp->assign(n, -1);
  for (int j = 0, b = 1; j < n; j++)
    if (j != rank) {
      (*sp)[b] = j;
      (*rp)[b] = j;
      b++;
    }
}
}  // namespace

bool flatEnabled(const ncclComm* comm) {
  return comm->ringFallback && comm->knobs.treeFlat && comm->nRanks > 1 && comm->nRanks <= kMaxReduceFusion;
}

size_t tableIndex(int group, int chan, int peer, int nRanks) {
  return ((size_t)group * kMaxChannels + chan) * nRanks + peer;
}

ncclResult_t transportPlan(ncclComm* comm) {
  const int n = comm->nRanks;
  for (int p = 0; p < 3; p++) {
    // a FIFO slot must stay far below the 2 GiB reach of a buffer descriptor (interpreter.h)
    if (comm->knobs.buffSizes[p] <= 0 || comm->knobs.buffSizes[p] > (1ll << 30)) {
      WARN("MSCCL: FIFO buffer size %lld (protocol %d) outside (0, 1 GiB]", (long long)comm->knobs.buffSizes[p], p);
      return ncclInvalidArgument;
    }
    comm->buffSizes[p] = (int)comm->knobs.buffSizes[p];
  }
  comm->llSlotLines = comm->buffSizes[kProtoLL] / kFifoSteps / 16;
  comm->simpleSlotBytes = comm->buffSizes[kProtoSimple] / kFifoSteps / 16 * 16;
  if (comm->llSlotLines < 128 || comm->simpleSlotBytes < 4096) {
    WARN("MSCCL: FIFO buffer sizes too small (LL %d, Simple %d)", comm->buffSizes[0], comm->buffSizes[2]);
    return ncclInvalidArgument;
  }
  if (comm->algos.size() > (size_t)kMaxAlgos) {
    WARN("MSCCL: %zu algorithms loaded, at most %d", comm->algos.size(), kMaxAlgos);
    return ncclInternalError;
  }
  comm->sendKeys.clear();
  comm->recvKeys.clear();
  for (size_t g = 0; g < comm->algos.size(); g++) {
    const Algorithm& a = comm->algos[g];
    std::map<std::pair<int, int>, int> seenS, seenR;
    for (int b = 0; b < a.nBlocks; b++) {
      const ThreadBlock& tb = a.tbs[b];
      if (tb.sendpeer >= 0) {
        auto k = std::make_pair((int)tb.channel, (int)tb.sendpeer);
        if (seenS.count(k)) {
          WARN("MSCCL: algorithm %s: thread blocks %d and %d both send to peer %d on channel %d",
               a.name.c_str(), seenS[k], b, tb.sendpeer, tb.channel);
          return ncclInvalidUsage;
        }
        seenS[k] = b;
        comm->sendKeys.push_back(ConnKey{(int)g, tb.channel, tb.sendpeer});
      }
      if (tb.recvpeer >= 0) {
        auto k = std::make_pair((int)tb.channel, (int)tb.recvpeer);
        if (seenR.count(k)) {
          WARN("MSCCL: algorithm %s: thread blocks %d and %d both receive from peer %d on channel %d",
               a.name.c_str(), seenR[k], b, tb.recvpeer, tb.channel);
          return ncclInvalidUsage;
        }
        seenR[k] = b;
        comm->recvKeys.push_back(ConnKey{(int)g, tb.channel, tb.recvpeer});
      }
    }
  }
  // ring fallback: ring channel c sends to rank+1 and receives from rank-1 (one sub-connection);
  // tree fallback: the chain's up / down thread blocks of channel c
  if (comm->ringFallback && n > 1) {
    for (int c = 0; c < kRingChannels; c++) {
      comm->sendKeys.push_back(ConnKey{kRingGroup, c, (comm->rank + 1) % n});
      comm->recvKeys.push_back(ConnKey{kRingGroup, c, (comm->rank + n - 1) % n});
    }
    std::vector<int> sp, rp;
    treePeers(comm->rank, n, &sp, &rp);
    for (int b = 0; b < 2 * kRingChannels; b++) {
      if (sp[b] >= 0) comm->sendKeys.push_back(ConnKey{kTreeGroup, b / 2, sp[b]});
      if (rp[b] >= 0) comm->recvKeys.push_back(ConnKey{kTreeGroup, b / 2, rp[b]});
    }
  }
  if (flatEnabled(comm))
    for (int p = 0; p < n; p++)
      if (p != comm->rank) {
        comm->sendKeys.push_back(ConnKey{kFlatGroup, 0, p});
        comm->recvKeys.push_back(ConnKey{kFlatGroup, 0, p});
      }
  // MSCCL_AMD_FIFO_PAD (bytes, rounded to 4 KiB; default 0): extra space after every FIFO, so
  // sub-connections do not start at the same offset modulo the FIFO size (a placement
  // experiment; each rank publishes its own strides, so ranks need not agree)
  const int64_t pad = (int64_t)alignUp((size_t)std::max<int64_t>(0, envInt("MSCCL_AMD_FIFO_PAD", 0)), kFifoAlign);
  const int64_t llBytes = (int64_t)alignUp((size_t)kLLFifoSlots * comm->llSlotLines * 16, kFifoAlign) + pad;
  const int64_t simpleBytes = (int64_t)alignUp((size_t)kFifoSteps * comm->simpleSlotBytes, kFifoAlign) + pad;
  comm->table.assign((size_t)kNumGroups * kMaxChannels * n,
                     PeerOffsets{-1, -1, -1, -1, llBytes, simpleBytes, (int64_t)kWordStride, 0});
  size_t off = 0;
  for (auto& k : comm->sendKeys) {
    comm->table[tableIndex(k.group, k.chan, k.peer, n)].sendHead = (int64_t)off;
    off += kWordStride * groupSubs(comm, k.group);
  }
  for (auto& k : comm->recvKeys) {
    comm->table[tableIndex(k.group, k.chan, k.peer, n)].recvTail = (int64_t)off;
    off += kWordStride * groupSubs(comm, k.group);
  }
  off = alignUp(off, kFifoAlign);
  for (auto& k : comm->recvKeys) {
    PeerOffsets& po = comm->table[tableIndex(k.group, k.chan, k.peer, n)];
    const uint8_t m = groupProtoMask(comm, k.group);
    const int subs = groupSubs(comm, k.group);
    if (m & ((1u << kProtoLL) | (1u << kProtoLL128))) {  // LL and LL128 share the LL FIFO memory
      po.recvLL = (int64_t)off;
      off += (size_t)llBytes * subs;
    }
    if (m & (1u << kProtoSimple)) {
      po.recvSimple = (int64_t)off;
      off += (size_t)simpleBytes * subs;
    }
  }
  comm->arenaSize = off ? off : kFifoAlign;
  hipError_t e = envInt("MSCCL_AMD_ARENA_COARSE", 0)
                     ? hipMalloc((void**)&comm->arena, comm->arenaSize)
                     : hipExtMallocWithFlags((void**)&comm->arena, comm->arenaSize, hipDeviceMallocUncached);
  if (e != hipSuccess) {
    WARN("MSCCL: cannot allocate %zu bytes of uncached transport memory: %s", comm->arenaSize, hipGetErrorString(e));
    return ncclUnhandledCudaError;
  }
  if (hipMemset(comm->arena, 0, comm->arenaSize) != hipSuccess) return ncclUnhandledCudaError;
  INFO(kSubInit | kSubP2P, "rank %d: %zu send / %zu recv connections, transport arena %zu bytes", comm->rank,
       comm->sendKeys.size(), comm->recvKeys.size(), comm->arenaSize);
  return ncclSuccess;
}

// Build and upload the slot-indexed connection records of one group: entry tb * subs + sub.
static ncclResult_t buildConns(ncclComm* comm, int group, int nTb, const std::vector<int>& sendPeer,
                               const std::vector<int>& recvPeer, const std::vector<int>& chan,
                               const std::vector<std::vector<PeerOffsets>>& tables, const std::vector<char*>& peerBases,
                               const std::vector<int>& peerRemote, DevSendConn** dS, DevRecvConn** dR) {
  const int n = comm->nRanks, me = comm->rank, S = groupSubs(comm, group);
  const uint8_t m = groupProtoMask(comm, group);
  // MSCCL_AMD_SIMPLE_FENCE=1: agent-scope fences around local Simple hand-offs too (a measurement
  // of what the fences would cost; the sc0 sc1 form needs none, interpreter.h: waitRecvTail)
  static const int localFence = envInt("MSCCL_AMD_SIMPLE_FENCE", 0) ? 2 : 0;
  const bool needLL = m & ((1u << kProtoLL) | (1u << kProtoLL128)), needS = m & (1u << kProtoSimple);
  std::vector<DevSendConn> hs((size_t)std::max(nTb, 1) * S);
  std::vector<DevRecvConn> hr((size_t)std::max(nTb, 1) * S);
  memset(hs.data(), 0, hs.size() * sizeof(DevSendConn));
  memset(hr.data(), 0, hr.size() * sizeof(DevRecvConn));
  for (int b = 0; b < nTb; b++) {
    if (sendPeer[b] >= 0) {
      const int p = sendPeer[b];
      const PeerOffsets& theirs = tables[p][tableIndex(group, chan[b], me, n)];
      const PeerOffsets& mine = comm->table[tableIndex(group, chan[b], p, n)];
      if (theirs.recvTail < 0 || (needLL && theirs.recvLL < 0) || (needS && theirs.recvSimple < 0)) {
        WARN("MSCCL: rank %d sends to rank %d on channel %d but rank %d has no matching receive", me, p, chan[b], p);
        return ncclInvalidUsage;
      }
      char* pb = peerBases[p];
      for (int s = 0; s < S; s++) {
        DevSendConn& c = hs[(size_t)b * S + s];
        c.ll = theirs.recvLL >= 0 ? (LLLine*)(pb + theirs.recvLL + s * theirs.llStride) : nullptr;
        c.simple = theirs.recvSimple >= 0 ? pb + theirs.recvSimple + s * theirs.simpleStride : nullptr;
        c.remoteTail = (uint64_t*)(pb + theirs.recvTail + s * theirs.wordStride);
        c.head = (uint64_t*)(comm->arena + mine.sendHead + s * mine.wordStride);
        c.llSlotLines = comm->llSlotLines;
        c.simpleSlotBytes = comm->simpleSlotBytes;
        c.remote = peerRemote[p] ? 1 : localFence;
      }
    }
    if (recvPeer[b] >= 0) {
      const int p = recvPeer[b];
      const PeerOffsets& theirs = tables[p][tableIndex(group, chan[b], me, n)];
      const PeerOffsets& mine = comm->table[tableIndex(group, chan[b], p, n)];
      if (theirs.sendHead < 0) {
        WARN("MSCCL: rank %d receives from rank %d on channel %d but rank %d has no matching send", me, p, chan[b],
             p);
        return ncclInvalidUsage;
      }
      for (int s = 0; s < S; s++) {
        DevRecvConn& c = hr[(size_t)b * S + s];
        c.ll = mine.recvLL >= 0 ? (LLLine*)(comm->arena + mine.recvLL + s * mine.llStride) : nullptr;
        c.simple = mine.recvSimple >= 0 ? comm->arena + mine.recvSimple + s * mine.simpleStride : nullptr;
        c.tail = (uint64_t*)(comm->arena + mine.recvTail + s * mine.wordStride);
        c.remoteHead = (uint64_t*)(peerBases[p] + theirs.sendHead + s * theirs.wordStride);
        c.llSlotLines = comm->llSlotLines;
        c.simpleSlotBytes = comm->simpleSlotBytes;
        c.remote = peerRemote[p] ? 1 : localFence;
      }
    }
  }
  if (hipMalloc(dS, hs.size() * sizeof(DevSendConn)) != hipSuccess) return ncclUnhandledCudaError;
  if (hipMalloc(dR, hr.size() * sizeof(DevRecvConn)) != hipSuccess) return ncclUnhandledCudaError;
  if (hipMemcpy(*dS, hs.data(), hs.size() * sizeof(DevSendConn), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(*dR, hr.data(), hr.size() * sizeof(DevRecvConn), hipMemcpyHostToDevice) != hipSuccess)
    return ncclUnhandledCudaError;
  return ncclSuccess;
}

ncclResult_t transportConnect(ncclComm* comm, const std::vector<std::vector<PeerOffsets>>& tables,
                              const std::vector<char*>& peerBases, const std::vector<int>& peerRemote) {
  const int n = comm->nRanks;
  comm->devAlgos.assign(comm->algos.size(), DevAlgoHost());
  for (size_t g = 0; g < comm->algos.size(); g++) {
    const Algorithm& a = comm->algos[g];
    std::vector<int> sp(a.nBlocks), rp(a.nBlocks), ch(a.nBlocks);
    for (int b = 0; b < a.nBlocks; b++) {
      sp[b] = a.tbs[b].sendpeer;
      rp[b] = a.tbs[b].recvpeer;
      ch[b] = a.tbs[b].channel;
    }
    DevAlgoHost& d = comm->devAlgos[g];
    d.connSplit = groupSubs(comm, (int)g);
    NCCLCHECK(buildConns(comm, (int)g, a.nBlocks, sp, rp, ch, tables, peerBases, peerRemote, &d.dSend, &d.dRecv));
  }
  if (comm->ringFallback && n > 1) {
    std::vector<int> sp(kRingChannels, (comm->rank + 1) % n), rp(kRingChannels, (comm->rank + n - 1) % n),
        ch(kRingChannels);
    for (int c = 0; c < kRingChannels; c++) ch[c] = c;
    NCCLCHECK(buildConns(comm, kRingGroup, kRingChannels, sp, rp, ch, tables, peerBases, peerRemote, &comm->ringSend,
                         &comm->ringRecv));
    std::vector<int> tsp, trp, tch(2 * kRingChannels);
    treePeers(comm->rank, n, &tsp, &trp);
    for (int b = 0; b < 2 * kRingChannels; b++) tch[b] = b / 2;
    NCCLCHECK(buildConns(comm, kTreeGroup, 2 * kRingChannels, tsp, trp, tch, tables, peerBases, peerRemote,
                         &comm->treeSend, &comm->treeRecv));
  }
  if (flatEnabled(comm)) {
    std::vector<int> fsp, frp, fch(n, 0);
    flatPeers(comm->rank, n, &fsp, &frp);
    NCCLCHECK(buildConns(comm, kFlatGroup, n, fsp, frp, fch, tables, peerBases, peerRemote, &comm->flatSend,
                         &comm->flatRecv));
  }
  return ncclSuccess;
}

// Thread-block image: [DevTbHeader][nsteps DevTransfer][ndeps int16 bid][ndeps int16 step]
// [nreds int16 source offsets], padded to 16 B.  Every image of a group has the same stride, so
// a workgroup finds its own from its block index (devcomm.h).
static void putImage(std::vector<char>& out, size_t at, const DevTbHeader& h, const std::vector<Transfer>& ts,
                     const std::vector<int16_t>& depBid, const std::vector<int16_t>& depStep,
                     const std::vector<int16_t>& reds) {
  char* p = out.data() + at;
  memcpy(p, &h, sizeof(h));
  p += sizeof(h);
  for (const Transfer& t : ts) {
    DevTransfer x;
    memset(&x, 0, sizeof(x));
    x.srcoff = t.srcoff;
    x.dstoff = t.dstoff;
    x.srcbuf = t.srcbuf;
    x.dstbuf = t.dstbuf;
    x.type = t.type;
    x.count = t.count;
    x.depPtr = t.depPtr;
    x.numDeps = t.numDeps;
    x.redPtr = t.redPtr;
    x.numReds = (uint8_t)t.numReds;
    x.hasDep = (uint8_t)t.hasDep;
    memcpy(p, &x, sizeof(x));
    p += sizeof(x);
  }
  for (const std::vector<int16_t>* v : {&depBid, &depStep, &reds}) {
    if (!v->empty()) memcpy(p, v->data(), v->size() * sizeof(int16_t));
    p += v->size() * sizeof(int16_t);
  }
}

static size_t imageBytes(size_t nsteps, size_t ndeps, size_t nreds) {
  return alignUp(sizeof(DevTbHeader) + nsteps * sizeof(DevTransfer) + (2 * ndeps + nreds) * sizeof(int16_t), 16);
}

static ncclResult_t uploadImages(const std::vector<char>& img, DevAlgoHost* d) {
  if (hipMalloc(&d->dImages, img.size()) != hipSuccess) return ncclUnhandledCudaError;
  if (hipMemcpy(d->dImages, img.data(), img.size(), hipMemcpyHostToDevice) != hipSuccess) return ncclUnhandledCudaError;
  return ncclSuccess;
}

// The reference's ring collectives as programs of this interpreter, one thread block per ring
// channel.  Offsets are indices, resolved per iteration by the kernel's ring mode:
//   AllReduce: chunk index c of calcOffset(c) (all_reduce.h:51-98);
//   ReduceScatter / AllGather: rank index d of chunkOffset + d * size, -1 = chunkOffset alone
//   (reduce_scatter.h:50-65, all_gather.h:52-75).
// Kinds: 0 AllReduce, 1 ReduceScatter, 2 AllGather in place, 3 AllGather out of place.
static std::vector<Transfer> ringProgram(int kind, int r, int n) {
  std::vector<Transfer> v;
  auto add = [&](uint8_t type, uint8_t sb, int so, uint8_t db, int dof) {
    Transfer t;
    t.type = type;
    t.srcbuf = sb;
    t.srcoff = (int16_t)so;
    t.dstbuf = db;
    t.dstoff = (int16_t)dof;
    t.count = 1;
    v.push_back(t);
  };
  auto ring = [&](int k) { return (r + k) % n; };  // devUserRanks of the rank-order ring
  if (kind == 0) {
    add(kSend, kInput, ring(n - 1), kInput, -1);
    for (int j = 2; j < n; j++) add(kRecvReduceSend, kInput, ring(n - j), kInput, -1);
    add(kRecvReduceCopySend, kInput, ring(0), kOutput, ring(0));
    for (int j = 1; j < n - 1; j++) add(kRecvCopySend, kInput, -1, kOutput, ring(n - j));
    add(kRecv, kInput, -1, kOutput, ring(1));
  } else if (kind == 1) {
    add(kSend, kInput, ring(n - 1), kInput, -1);
    for (int j = 2; j < n; j++) add(kRecvReduceSend, kInput, ring(n - j), kInput, -1);
    add(kRecvReduceCopy, kInput, ring(0), kOutput, -1);
  } else {
    if (kind == 2) add(kSend, kOutput, ring(0), kOutput, -1);  // directSend from the output
    else add(kCopySend, kInput, -1, kOutput, ring(0));          // directCopySend
    for (int j = 1; j < n - 1; j++) add(kRecvCopySend, kInput, -1, kOutput, ring(n - j));
    add(kRecv, kInput, -1, kOutput, ring(1));
  }
  return v;
}

ncclResult_t ringUpload(ncclComm* comm) {
  const int n = comm->nRanks;
  if (!comm->ringFallback || n < 2) return ncclSuccess;
  const std::vector<int16_t> none;
  for (int kind = 0; kind < 4; kind++) {
    const std::vector<Transfer> prog = ringProgram(kind, comm->rank, n);
    DevAlgoHost& d = comm->ringAlgos[kind];
    d.nBlocks = kRingChannels;
    d.tbStride = (int)imageBytes(prog.size(), 0, 0);
    d.connSplit = 1;
    d.dSend = comm->ringSend;  // owned by the communicator, shared by the four ring programs
    d.dRecv = comm->ringRecv;
    std::vector<char> img((size_t)d.tbStride * kRingChannels, 0);
    for (int c = 0; c < kRingChannels; c++) {  // every channel runs the same program
      DevTbHeader h;
      memset(&h, 0, sizeof(h));
      h.hasSend = h.hasRecv = 1;
      h.nsteps = (uint16_t)prog.size();
      putImage(img, (size_t)c * d.tbStride, h, prog, none, none, none);
    }
    NCCLCHECK(uploadImages(img, &d));
  }
  {
    // tree AllReduce (all_reduce.h:103-298, split form): offsets are -1 = the chunk offset
    const int r = comm->rank;
    std::vector<int> sp, rp;
    treePeers(r, n, &sp, &rp);
    auto one = [](uint8_t type, uint8_t sb, uint8_t db) {
      Transfer t;
      t.type = type;
      t.srcbuf = sb;
      t.srcoff = -1;
      t.dstbuf = db;
      t.dstoff = -1;
      t.count = 1;
      return std::vector<Transfer>{t};
    };
    std::vector<Transfer> up, down;
    if (r == 0) up = one(kRecvReduceCopySend, kInput, kOutput);   // recv child, reduce, result down
    else if (r == n - 1) up = one(kSend, kInput, kInput);         // leaf: send up
    else up = one(kRecvReduceSend, kInput, kInput);               // recv child, reduce, send up
    if (r == n - 1) down = one(kRecv, kInput, kOutput);           // leaf: receive the result
    else if (r > 0) down = one(kRecvCopySend, kInput, kOutput);   // receive, keep, pass down
    DevAlgoHost& d = comm->ringAlgos[4];
    d.nBlocks = 2 * kRingChannels;
    d.tbStride = (int)imageBytes(1, 0, 0);
    d.connSplit = 1;
    d.dSend = comm->treeSend;
    d.dRecv = comm->treeRecv;
    std::vector<char> img((size_t)d.tbStride * d.nBlocks, 0);
    for (int b = 0; b < d.nBlocks; b++) {
      const std::vector<Transfer>& prog = (b & 1) ? down : up;
      DevTbHeader h;
      memset(&h, 0, sizeof(h));
      h.hasSend = sp[b] >= 0;
      h.hasRecv = rp[b] >= 0;
      h.nsteps = (uint16_t)prog.size();
      putImage(img, (size_t)b * d.tbStride, h, prog, none, none, none);
    }
    NCCLCHECK(uploadImages(img, &d));
  }
  if (flatEnabled(comm)) {
    // The flat forms (plan.cc: makeFlatTreePlan), run by mscclFoldKernel (interpreter.h:
    // runFold): each rank exchanges with every peer p_j over the flat connections of thread block
    // 1 + j (flatPeers) in one hop.  The AllReduce folds every rank's input in the order x_{n-1},
    // ..., x_0: acc = x_{n-1}, acc = fn(acc, x_q) for q = n - 2 down to 0, the chain tree's fold
    // (runTreeSplit on the chain, transport.cc: treePeers: leaf n - 1 sends its input up, rank q
    // folds fn(child's partial, x_q), the root's result comes back down).  Every op admitted (Sum,
    // Prod, Max, Min) is commutative per element, so the values are the tree's bit for bit,
    // whatever side of fn each operand sits on; the same holds for the ReduceScatter's ring order.
    // No scratch, no dependency flag, no copy.
    const int r = comm->rank;
    std::vector<int> sp, rp;
    flatPeers(r, n, &sp, &rp);
    // Three tables in the image's reduction list, one transfer each:
    //   0: the AllReduce fold order (thread block per position, ranks n-1 .. 0, -1 = own input);
    //   1: the ReduceScatter fold order, the ring's for this rank's block (reduce_scatter.h:13-67:
    //      the block starts at rank r+1 and is reduced at r+2, ..., r+n-1, then here): ranks r+1,
    //      ..., r+n-1, then the own input;
    //   2: the rank each peer record k (thread block k + 1) connects, then this rank.
    auto tbOf = [&](int q) {
      for (int b = 1; b < n; b++)
        if (rp[b] == q) return b;
      return -1;
    };
    // The AllReduce's fold orders (ranks): the flat tree's is n-1 .. 0 (one class); a lowered
    // schedule's are its own (lower.cc), one per class of chunks.  Tables in the image's reduction
    // list, one transfer each (positions map to peer records, -1 = this rank's input):
    //   0: the AllReduce fold order of class 0; 1: the ReduceScatter order; 2: the rank of every
    //   peer record, then this rank; with several classes (or a two-phase form) also 3: every
    //   class's order (srcoff = classes) and 4: the class of every chunk (srcoff = chunks); with a
    //   two-phase form (lower.h) also 5: the chunks each rank owns, ascending, per peer record and
    //   then this rank's (srcoff = chunks per rank; interpreter.h: runTwoPhase).
    auto foldImage = [&](const ncclComm::FoldProgram& fp, DevAlgoHost& d) -> ncclResult_t {
    std::vector<int16_t> reds;
    const std::vector<int>& arOrder = fp.order[0];
    for (int q : arOrder) reds.push_back((int16_t)(q == r ? -1 : tbOf(q)));
    for (int i = 1; i <= n; i++) {
      const int q = (r + i) % n;
      reds.push_back((int16_t)(q == r ? -1 : tbOf(q)));
    }
    for (int b = 1; b < n; b++) reds.push_back((int16_t)rp[b]);
    reds.push_back((int16_t)r);
    const bool two = !fp.owner.empty();
    const bool multi = fp.order.size() > 1 || two;
    std::vector<Transfer> ts(two ? 6 : multi ? 5 : 3);
    for (int i = 0; i < 3; i++) {
      ts[i].type = kFoldRecv;
      ts[i].srcbuf = kInput;
      ts[i].dstbuf = kOutput;
      ts[i].count = 1;
      ts[i].numReds = (int16_t)n;
      ts[i].redPtr = (int16_t)(i * n);
    }
    if (multi) {
      ts[3] = ts[0];
      ts[3].redPtr = (int16_t)reds.size();
      ts[3].srcoff = (int16_t)fp.order.size();
      for (const std::vector<int>& o : fp.order)
        for (int q : o) reds.push_back((int16_t)(q == r ? -1 : tbOf(q)));
      ts[4] = ts[0];
      ts[4].redPtr = (int16_t)reds.size();
      ts[4].srcoff = (int16_t)fp.chunkClass.size();
      for (int k : fp.chunkClass) reds.push_back((int16_t)k);
    }
    if (two) {
      const int K = (int)fp.owner.size() / n;
      ts[5] = ts[0];
      ts[5].redPtr = (int16_t)reds.size();
      ts[5].srcoff = (int16_t)K;
      auto list = [&](int q) {
        for (int c = 0; c < (int)fp.owner.size(); c++)
          if (fp.owner[c] == q) reds.push_back((int16_t)c);
      };
      for (int b = 1; b < n; b++) list(rp[b]);
      list(r);
    }
    if (imageBytes(ts.size(), 0, reds.size()) > (size_t)kMaxImage16 * 16) {  // the kernel's LDS copy (BlockShared::img)
      WARN("MSCCL: the fold program of %d chunks does not fit a workgroup's image", (int)fp.chunkClass.size());
      return ncclInternalError;
    }
    d.nBlocks = 1;
    d.tbStride = (int)imageBytes(ts.size(), 0, reds.size());
    d.connSplit = comm->flatSubs;
    d.dSend = comm->flatSend;
    d.dRecv = comm->flatRecv;
    std::vector<char> img((size_t)d.tbStride, 0);
    DevTbHeader h;
    memset(&h, 0, sizeof(h));
    h.nsteps = (uint16_t)ts.size();
    h.nreds = (uint16_t)reds.size();
    const std::vector<int16_t> none;
    putImage(img, 0, h, ts, none, none, reds);
    return uploadImages(img, &d);
    };
    ncclComm::FoldProgram chain;
    chain.order.emplace_back();
    for (int q = n - 1; q >= 0; q--) chain.order[0].push_back(q);
    NCCLCHECK(foldImage(chain, comm->ringAlgos[5]));
    // the one-hop MSCCL schedules (lower.cc): the fold with the schedule's orders, over the same
    // flat connections (the step counters are the connections', whichever program runs)
    comm->foldAlgos.assign(comm->algos.size(), DevAlgoHost());
    for (size_t g = 0; g < comm->algoFold.size(); g++)
      if (!comm->algoFold[g].order.empty()) NCCLCHECK(foldImage(comm->algoFold[g], comm->foldAlgos[g]));
  }
  return ncclSuccess;
}

// Longest run of chunks a thread block sends before it next receives (merge bound, devcomm.h).
int algoSendRunOf(const Algorithm& a) {
  int best = 0;
  for (int b = 0; b < a.nBlocks; b++) {
    int run = 0;
    for (const Transfer& t : a.tbs[b].transfers) {
      if (t.type == kSend) run += t.count;
      else if (t.type == kRecv || t.type == kRecvCopySend || t.type == kRecvReduceSend ||
               t.type == kRecvReduceCopy || t.type == kRecvReduceCopySend) run = 0;
      best = std::max(best, run);
    }
  }
  return best;
}

// Thread blocks whose first FIFO transfers are `s` then `rrc` of the same source chunks with a
// single peer (send peer == receive peer), with no flag published after the send and no wait
// before the receive.  When the peer's thread block on that connection has the same shape, the
// two ends exchange in lockstep: each FIFO step is sent, then the peer's same step is received
// and reduced with the values just sent, so the source is read once (LL: 7 S -> 6 S HBM bytes per
// rank for the pair exchange).  Each receive waits only for a step its peer sends before waiting
// itself, so the fused pair cannot deadlock, and an end that runs the pair unfused (s fully,
// then rrc) still makes progress against a fused one.  Values are those of s then rrc: the same
// fn(peer, local) per element (interpreter.h: llStep FUSED).
std::vector<FuseCandidate> fusableTbs(const Algorithm& a) {
  std::vector<FuseCandidate> out;
  auto fifo = [](uint8_t t) { return t <= kRecvReduceCopySend || t == kCopySend; };
  for (int b = 0; b < a.nBlocks; b++) {
    const ThreadBlock& tb = a.tbs[b];
    if (tb.sendpeer < 0 || tb.sendpeer != tb.recvpeer) continue;
    const std::vector<Transfer>& ts = tb.transfers;
    size_t i = 0;
    while (i < ts.size() && !fifo(ts[i].type)) i++;
    if (i + 1 >= ts.size()) continue;
    const Transfer &s = ts[i], &r = ts[i + 1];
    if (s.type == kSend && r.type == kRecvReduceCopy && s.srcbuf == r.srcbuf && s.srcoff == r.srcoff &&
        s.count == r.count && s.hasDep == 0 && r.numDeps == 0)
      out.push_back({(int16_t)b, (int16_t)i, (int16_t)tb.channel, tb.sendpeer});
  }
  return out;
}

// Transfers i, i + 1 of a program are an `s` and a `cpy` of the same source chunks that one
// copy-send pass may replace: no flag published between them, and the copy's destination chunks
// either are its source chunks (a self-copy writes back the values it read) or share none with
// them, so the bytes sent never depend on the order of the pass's loads and stores (the unfused
// s sends the source before the cpy writes).  Buffers i and o alias in an in-place call (the
// same memory for AllReduce, one block of it for ReduceScatter / AllGather), so there i and o
// count as one buffer for AllReduce and a cpy between them is not fused for the others.
bool sendCopyFusable(const Algorithm& a, const std::vector<Transfer>& ts, size_t i) {
  if (i + 1 >= ts.size()) return false;
  const Transfer &s = ts[i], &c = ts[i + 1];
  if (s.type != kSend || c.type != kLocalCopy || s.srcbuf != c.srcbuf || s.srcoff != c.srcoff ||
      s.count != c.count || s.hasDep != 0 || c.numDeps != 0)
    return false;
  const bool io = c.srcbuf != kScratch && c.dstbuf != kScratch;
  bool sameBuf = c.srcbuf == c.dstbuf;
  if (!sameBuf && a.inPlace && io) {
    if (a.coll != kAllReduce) return false;
    sameBuf = true;
  }
  if (!sameBuf) return true;
  const int s0 = c.srcoff, s1 = c.srcoff + c.count, d0 = c.dstoff, d1 = c.dstoff + c.count;
  return (s0 == d0) || s1 <= d0 || d1 <= s0;
}

// The pair form (the pair kernel, interpreter.h: PairRunner): every thread block runs exactly one
// fused exchange (listed in `fused`) of one input chunk at an affine chunk index, its rrc reading
// that chunk and writing the same index of the input or output, no dependency.
ncclComm::PairForm pairFormOf(const Algorithm& a, const std::vector<FuseCandidate>& fused) {
  ncclComm::PairForm pf;
  bool pair = a.nBlocks > 0;
  for (int b = 0; pair && b < a.nBlocks; b++) {
    const std::vector<Transfer>& ts = a.tbs[b].transfers;
    bool f = false;
    for (const FuseCandidate& c : fused) f |= c.tb == b && c.index == 0;
    pair = f && ts.size() == 2 && ts[0].type == kSend && ts[1].type == kRecvReduceCopy && ts[0].count == 1 &&
           ts[1].count == 1 && ts[0].srcbuf == 0 && ts[1].srcbuf == 0 && ts[1].srcoff == ts[0].srcoff &&
           ts[1].dstbuf <= 1 && ts[0].numDeps == 0 && ts[1].numDeps == 0 && ts[0].hasDep == 0 && ts[1].hasDep == 0;
    if (!pair) break;
    if (b == 0) {
      pf.src = ts[0].srcoff;
      pf.dst = ts[1].dstoff;
      pf.dstBuf = ts[1].dstbuf;
    } else if (b == 1) {
      pf.stride = ts[0].srcoff - pf.src;
    }
    pair = ts[0].srcoff == pf.src + b * pf.stride && ts[1].dstoff == pf.dst + b * pf.stride && ts[1].dstbuf == pf.dstBuf;
  }
  // RankWork carries src, dst and stride as int16: every one of them, and the last thread block's
  // chunk indices, must fit (the indices are affine in b, so the first and last bound them all)
  auto fits = [](int64_t x) { return x >= 0 && x < 32767; };
  const int64_t last = (int64_t)std::max(0, a.nBlocks - 1) * pf.stride;
  const bool ok = pair && fits(pf.src) && fits(pf.dst) && pf.stride >= -32767 && pf.stride < 32767 &&
                  fits(pf.src + last) && fits(pf.dst + last);
  return ok ? pf : ncclComm::PairForm();
}

// Pack every algorithm's per-tb programs into fixed-stride images and upload them (replaces
// the 29 MB mscclDevCommInfo copy of devCommSetup, init.cc:300-304).
ncclResult_t algoUpload(ncclComm* comm) {
  comm->algoSet.assign(comm->algos.size(), kSetAll);
  for (size_t g = 0; g < comm->algos.size(); g++) {
    // the small kernel variant its programs need (devcomm.h: kSetAll / kSetExchange)
    bool exchangeOnly = true;
    const Algorithm& a = comm->algos[g];
    if (g >= comm->devAlgos.size()) comm->devAlgos.resize(g + 1);
    DevAlgoHost& d = comm->devAlgos[g];
    d.nBlocks = a.nBlocks;
    size_t stride = 16;
    for (int b = 0; b < a.nBlocks; b++) {
      const ThreadBlock& tb = a.tbs[b];
      stride = std::max(stride, imageBytes(tb.transfers.size(), tb.depBid.size(), tb.redSrcOff.size()));
    }
    d.tbStride = (int)stride;
    std::vector<char> img(stride * std::max(a.nBlocks, 1), 0);
    for (int b = 0; b < a.nBlocks; b++) {
      const ThreadBlock& tb = a.tbs[b];
      DevTbHeader h;
      memset(&h, 0, sizeof(h));
      h.hasSend = tb.sendpeer >= 0;
      h.hasRecv = tb.recvpeer >= 0;
      h.nsteps = tb.nsteps;
      h.ndeps = (uint16_t)tb.depBid.size();
      h.nreds = (uint16_t)tb.redSrcOff.size();
      std::vector<Transfer> ts = tb.transfers;
      if (g < comm->algoFuse.size())
        for (const FuseCandidate& f : comm->algoFuse[g])
          if (f.tb == b) ts[f.index].type = kSendRecvReduceCopy;
      // s followed by a cpy of the same source chunks (an out-of-place AllGather's own block):
      // one copy-send pass reads the source once.  A local change: the FIFO steps are the s's.
      for (size_t i = 0; comm->knobs.fuse && i + 1 < ts.size(); i++)
        if (sendCopyFusable(a, ts, i)) ts[i].type = kSendCopy;
      for (const Transfer& t : ts)
        if (t.type != kSend && t.type != kRecvReduceCopy && t.type != kSendRecvReduceCopy) exchangeOnly = false;
      putImage(img, (size_t)b * stride, h, ts, tb.depBid, tb.depStep, tb.redSrcOff);
    }
    comm->algoSet[g] = exchangeOnly ? kSetExchange : kSetAll;
    if (g >= comm->algoPair.size()) comm->algoPair.resize(g + 1);
    comm->algoPair[g] = exchangeOnly && g < comm->algoFuse.size() ? pairFormOf(a, comm->algoFuse[g]) : ncclComm::PairForm();
    NCCLCHECK(uploadImages(img, &d));
  }
  // the direct forms' programs (interpreter.h: DirectRunner): transfer 0 lists this rank's fold
  // order (ranks) per class (srcoff = classes), transfer 1 every output chunk's class (srcoff =
  // chunks); the AllGather needs none
  comm->directAlgos.assign(comm->algos.size(), DevAlgoHost());
  for (size_t g = 0; g < comm->algoDirect.size() && g < comm->algos.size(); g++) {
    const ncclComm::DirectProgram& dp = comm->algoDirect[g];
    if (dp.coll < 0 || dp.coll == kAllGather) continue;
    std::vector<int16_t> reds;
    std::vector<Transfer> ts(2);
    ts[0].srcoff = (int16_t)dp.order.size();
    ts[0].redPtr = 0;
    for (const std::vector<int>& o : dp.order)
      for (int q : o) reds.push_back((int16_t)q);
    ts[1].srcoff = (int16_t)dp.chunkClass.size();
    ts[1].redPtr = (int16_t)reds.size();
    for (int k : dp.chunkClass) reds.push_back((int16_t)k);
    DevAlgoHost& d = comm->directAlgos[g];
    d.nBlocks = 1;
    d.tbStride = (int)imageBytes(ts.size(), 0, reds.size());  // read from global memory (DirectShared tables)
    std::vector<char> img((size_t)d.tbStride, 0);
    DevTbHeader h;
    memset(&h, 0, sizeof(h));
    h.nsteps = (uint16_t)ts.size();
    h.nreds = (uint16_t)reds.size();
    const std::vector<int16_t> none;
    putImage(img, 0, h, ts, none, none, reds);
    NCCLCHECK(uploadImages(img, &d));
  }
  // the ring fallback's ReduceScatter (plan.cc: planCall): block b of the output is folded along
  // the ring from rank b + 1 (its first `s`) to b (its `rrc`), reduce_scatter.h:50-65 with the ring
  // in rank order; every chunk of the block alike, so one class and one chunk
  if (comm->knobs.direct && comm->clique != 0) {
    std::vector<int16_t> reds;
    std::vector<Transfer> ts(2);
    ts[0].srcoff = 1;
    ts[0].redPtr = 0;
    for (int j = 1; j <= comm->nRanks; j++) reds.push_back((int16_t)((comm->rank + j) % comm->nRanks));
    ts[1].srcoff = 1;
    ts[1].redPtr = (int16_t)reds.size();
    reds.push_back(0);
    DevAlgoHost& d = comm->ringDirectRS;
    d.nBlocks = 1;
    d.tbStride = (int)imageBytes(ts.size(), 0, reds.size());
    std::vector<char> img((size_t)d.tbStride, 0);
    DevTbHeader h;
    memset(&h, 0, sizeof(h));
    h.nsteps = (uint16_t)ts.size();
    h.nreds = (uint16_t)reds.size();
    const std::vector<int16_t> none;
    putImage(img, 0, h, ts, none, none, reds);
    NCCLCHECK(uploadImages(img, &d));
  }
  return ringUpload(comm);
}

}  // namespace msccl

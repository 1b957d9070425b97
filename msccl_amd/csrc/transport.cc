// xGMI peer transport for MSCCL connections.
//
// Replaces the reference's P2P transport (transport/p2p.cc:143-344) and the MSCCL connect block
// of initTransportsRank (init.cc:781-874):
//   * one connection per (channel, peer) and direction, as named by the XML thread blocks;
//   * the receiver owns the FIFOs (LL: 8 steps x 4096 16-B lines; Simple: 8 x 512 KiB by
//     default, NCCL_LL_BUFFSIZE / NCCL_BUFFSIZE override) and a tail word; the sender owns a
//     head word the receiver writes.  All of it lives in one uncached (fine-grained) HBM arena
//     per rank, exported once per rank (hipIpc) or shared by pointer inside a process;
//   * a rank's layout is published as a table [channel][peer] -> offsets and exchanged.
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
}  // namespace

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
  std::map<ConnKey, uint8_t> sends, recvs;
  for (auto& a : comm->algos) {
    std::map<ConnKey, int> seenS, seenR;
    for (int b = 0; b < a.nBlocks; b++) {
      const ThreadBlock& tb = a.tbs[b];
      uint8_t bit = (uint8_t)(1u << a.proto);
      if (tb.sendpeer >= 0) {
        ConnKey k{tb.channel, tb.sendpeer};
        if (seenS.count(k)) {
          WARN("MSCCL: algorithm %s: thread blocks %d and %d both send to peer %d on channel %d",
               a.name.c_str(), seenS[k], b, tb.sendpeer, tb.channel);
          return ncclInvalidUsage;
        }
        seenS[k] = b;
        sends[k] |= bit;
      }
      if (tb.recvpeer >= 0) {
        ConnKey k{tb.channel, tb.recvpeer};
        if (seenR.count(k)) {
          WARN("MSCCL: algorithm %s: thread blocks %d and %d both receive from peer %d on channel %d",
               a.name.c_str(), seenR[k], b, tb.recvpeer, tb.channel);
          return ncclInvalidUsage;
        }
        seenR[k] = b;
        recvs[k] |= bit;
      }
    }
  }
  // ring fallback connections: one ring per channel kRingChanBase + c (send to rank+1, receive
  // from rank-1), LL and Simple FIFOs, one sub-connection each (the ring runs unsplit)
  if (comm->ringFallback && n > 1) {
    const uint8_t bits = (uint8_t)((1u << kProtoLL) | (1u << kProtoSimple));
    for (int c = 0; c < kRingChannels; c++) {
      sends[ConnKey{kRingChanBase + c, (comm->rank + 1) % n}] |= bits;
      recvs[ConnKey{kRingChanBase + c, (comm->rank + n - 1) % n}] |= bits;
    }
  }
  comm->sendKeys.clear();
  comm->recvKeys.clear();
  comm->sendProtoMask.clear();
  comm->recvProtoMask.clear();
  for (auto& kv : sends) { comm->sendKeys.push_back(kv.first); comm->sendProtoMask.push_back(kv.second); }
  for (auto& kv : recvs) { comm->recvKeys.push_back(kv.first); comm->recvProtoMask.push_back(kv.second); }

  const int S = comm->maxSplit;
  const int64_t llBytes = (int64_t)alignUp((size_t)kLLFifoSlots * comm->llSlotLines * 16, kFifoAlign);
  const int64_t simpleBytes = (int64_t)alignUp((size_t)kFifoSteps * comm->simpleSlotBytes, kFifoAlign);
  comm->table.assign((size_t)kTableChannels * n, PeerOffsets{-1, -1, -1, -1, llBytes, simpleBytes, (int64_t)kWordStride, 0});
  // ring keys have a single sub-connection: stride 0 makes every sub alias sub 0
  auto subsOf = [&](const ConnKey& k) { return k.chan >= kRingChanBase ? 1 : S; };
  for (int c = kRingChanBase; c < kTableChannels; c++)
    for (int p = 0; p < n; p++) {
      PeerOffsets& po = comm->table[(size_t)c * n + p];
      po.llStride = po.simpleStride = po.wordStride = 0;
    }
  size_t off = 0;
  for (auto& k : comm->sendKeys) { comm->table[(size_t)k.chan * n + k.peer].sendHead = (int64_t)off; off += kWordStride * subsOf(k); }
  for (auto& k : comm->recvKeys) { comm->table[(size_t)k.chan * n + k.peer].recvTail = (int64_t)off; off += kWordStride * subsOf(k); }
  off = alignUp(off, kFifoAlign);
  for (size_t i = 0; i < comm->recvKeys.size(); i++) {
    auto& k = comm->recvKeys[i];
    PeerOffsets& po = comm->table[(size_t)k.chan * n + k.peer];
    // LL and LL128 share the LL FIFO memory (two line formats)
    if (comm->recvProtoMask[i] & ((1u << kProtoLL) | (1u << kProtoLL128))) {
      po.recvLL = (int64_t)off;
      off += (size_t)llBytes * subsOf(k);
    }
    if (comm->recvProtoMask[i] & (1u << kProtoSimple)) {
      po.recvSimple = (int64_t)off;
      off += (size_t)simpleBytes * subsOf(k);
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

ncclResult_t transportConnect(ncclComm* comm, const std::vector<std::vector<PeerOffsets>>& tables,
                              const std::vector<char*>& peerBases, const std::vector<int>& peerRemote) {
  const int n = comm->nRanks, me = comm->rank, S = comm->maxSplit;
  std::vector<DevSendConn> hs(comm->sendKeys.size() * S);
  std::vector<DevRecvConn> hr(comm->recvKeys.size() * S);
  for (size_t i = 0; i < comm->sendKeys.size(); i++) {
    const ConnKey& k = comm->sendKeys[i];
    const PeerOffsets& theirs = tables[k.peer][(size_t)k.chan * n + me];
    const PeerOffsets& mine = comm->table[(size_t)k.chan * n + k.peer];
    uint8_t need = comm->sendProtoMask[i];
    bool needLL = need & ((1u << kProtoLL) | (1u << kProtoLL128)), needS = need & (1u << kProtoSimple);
    if (theirs.recvTail < 0 || (needLL && theirs.recvLL < 0) || (needS && theirs.recvSimple < 0)) {
      WARN("MSCCL: rank %d sends to rank %d on channel %d but rank %d has no matching receive", me, k.peer,
           k.chan, k.peer);
      return ncclInvalidUsage;
    }
    char* pb = peerBases[k.peer];
    for (int s = 0; s < S; s++) {
      DevSendConn& c = hs[i * S + s];
      memset(&c, 0, sizeof(c));
      c.ll = theirs.recvLL >= 0 ? (LLLine*)(pb + theirs.recvLL + s * theirs.llStride) : nullptr;
      c.simple = theirs.recvSimple >= 0 ? pb + theirs.recvSimple + s * theirs.simpleStride : nullptr;
      c.remoteTail = (uint64_t*)(pb + theirs.recvTail + s * theirs.wordStride);
      c.head = (uint64_t*)(comm->arena + mine.sendHead + s * mine.wordStride);
      c.step = 0;
      c.llSlotLines = comm->llSlotLines;
      c.simpleSlotBytes = comm->simpleSlotBytes;
      c.remote = peerRemote[k.peer];
    }
  }
  for (size_t i = 0; i < comm->recvKeys.size(); i++) {
    const ConnKey& k = comm->recvKeys[i];
    const PeerOffsets& theirs = tables[k.peer][(size_t)k.chan * n + me];
    const PeerOffsets& mine = comm->table[(size_t)k.chan * n + k.peer];
    if (theirs.sendHead < 0) {
      WARN("MSCCL: rank %d receives from rank %d on channel %d but rank %d has no matching send", me, k.peer,
           k.chan, k.peer);
      return ncclInvalidUsage;
    }
    for (int s = 0; s < S; s++) {
      DevRecvConn& c = hr[i * S + s];
      memset(&c, 0, sizeof(c));
      c.ll = mine.recvLL >= 0 ? (LLLine*)(comm->arena + mine.recvLL + s * mine.llStride) : nullptr;
      c.simple = mine.recvSimple >= 0 ? comm->arena + mine.recvSimple + s * mine.simpleStride : nullptr;
      c.tail = (uint64_t*)(comm->arena + mine.recvTail + s * mine.wordStride);
      c.remoteHead = (uint64_t*)(peerBases[k.peer] + theirs.sendHead + s * theirs.wordStride);
      c.step = 0;
      c.llSlotLines = comm->llSlotLines;
      c.simpleSlotBytes = comm->simpleSlotBytes;
    }
  }
  if (!hs.empty()) {
    if (hipMalloc(&comm->dSend, hs.size() * sizeof(DevSendConn)) != hipSuccess) return ncclUnhandledCudaError;
    hipMemcpy(comm->dSend, hs.data(), hs.size() * sizeof(DevSendConn), hipMemcpyHostToDevice);
  }
  if (!hr.empty()) {
    if (hipMalloc(&comm->dRecv, hr.size() * sizeof(DevRecvConn)) != hipSuccess) return ncclUnhandledCudaError;
    hipMemcpy(comm->dRecv, hr.data(), hr.size() * sizeof(DevRecvConn), hipMemcpyHostToDevice);
  }
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
  int sendIdx[kRingChannels], recvIdx[kRingChannels];
  for (int c = 0; c < kRingChannels; c++) {
    sendIdx[c] = recvIdx[c] = -1;
    for (size_t i = 0; i < comm->sendKeys.size(); i++)
      if (comm->sendKeys[i] == ConnKey{kRingChanBase + c, (comm->rank + 1) % n}) sendIdx[c] = (int)i;
    for (size_t i = 0; i < comm->recvKeys.size(); i++)
      if (comm->recvKeys[i] == ConnKey{kRingChanBase + c, (comm->rank + n - 1) % n}) recvIdx[c] = (int)i;
    if (sendIdx[c] < 0 || recvIdx[c] < 0) return ncclInternalError;
  }
  for (int kind = 0; kind < 4; kind++) {
    const std::vector<Transfer> prog = ringProgram(kind, comm->rank, n);
    std::vector<DevTbHeader> hdr(kRingChannels);
    std::vector<char> blob;
    for (const Transfer& t : prog) {
      DevTransfer x;
      memset(&x, 0, sizeof(x));
      x.srcoff = t.srcoff;
      x.dstoff = t.dstoff;
      x.srcbuf = t.srcbuf;
      x.dstbuf = t.dstbuf;
      x.type = t.type;
      x.count = t.count;
      const char* p = (const char*)&x;
      blob.insert(blob.end(), p, p + sizeof(x));
    }
    blob.resize(alignUp(blob.size() + 16, 16));
    for (int c = 0; c < kRingChannels; c++) {  // every channel runs the same program
      DevTbHeader& h = hdr[c];
      memset(&h, 0, sizeof(h));
      h.sendConn = (int16_t)sendIdx[c];
      h.recvConn = (int16_t)recvIdx[c];
      h.nsteps = (uint16_t)prog.size();
      h.blobOffset = 0;
    }
    DevAlgoHost& d = comm->ringAlgos[kind];
    d.nBlocks = kRingChannels;
    if (hipMalloc(&d.dTbs, hdr.size() * sizeof(DevTbHeader)) != hipSuccess) return ncclUnhandledCudaError;
    if (hipMalloc(&d.dBlob, blob.size()) != hipSuccess) return ncclUnhandledCudaError;
    hipMemcpy(d.dTbs, hdr.data(), hdr.size() * sizeof(DevTbHeader), hipMemcpyHostToDevice);
    hipMemcpy(d.dBlob, blob.data(), blob.size(), hipMemcpyHostToDevice);
  }
  return ncclSuccess;
}

// Pack every algorithm's per-tb programs and upload them (replaces the 29 MB
// mscclDevCommInfo copy of devCommSetup, init.cc:300-304).
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

ncclResult_t algoUpload(ncclComm* comm) {
  comm->devAlgos.clear();
  for (auto& a : comm->algos) {
    DevAlgoHost d;
    d.nBlocks = a.nBlocks;
    std::vector<DevTbHeader> hdr(a.nBlocks > 0 ? a.nBlocks : 1);
    std::vector<char> blob;
    for (int b = 0; b < a.nBlocks; b++) {
      const ThreadBlock& tb = a.tbs[b];
      DevTbHeader& h = hdr[b];
      memset(&h, 0, sizeof(h));
      h.sendConn = h.recvConn = -1;
      for (size_t i = 0; i < comm->sendKeys.size(); i++)
        if (tb.sendpeer >= 0 && comm->sendKeys[i] == ConnKey{tb.channel, tb.sendpeer}) h.sendConn = (int16_t)i;
      for (size_t i = 0; i < comm->recvKeys.size(); i++)
        if (tb.recvpeer >= 0 && comm->recvKeys[i] == ConnKey{tb.channel, tb.recvpeer}) h.recvConn = (int16_t)i;
      h.nsteps = tb.nsteps;
      h.ndeps = (uint16_t)tb.depBid.size();
      h.nreds = (uint16_t)tb.redSrcOff.size();
      size_t start = alignUp(blob.size(), 16);
      blob.resize(start);
      h.blobOffset = (uint32_t)start;
      for (const Transfer& t : tb.transfers) {
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
        const char* p = (const char*)&x;
        blob.insert(blob.end(), p, p + sizeof(x));
      }
      auto put16 = [&](const std::vector<int16_t>& v) {
        const char* p = (const char*)v.data();
        blob.insert(blob.end(), p, p + v.size() * sizeof(int16_t));
      };
      put16(tb.depBid);
      put16(tb.depStep);
      put16(tb.redSrcOff);
    }
    blob.resize(alignUp(blob.size() + 16, 16));
    if (hipMalloc(&d.dTbs, hdr.size() * sizeof(DevTbHeader)) != hipSuccess) return ncclUnhandledCudaError;
    if (hipMalloc(&d.dBlob, blob.size()) != hipSuccess) return ncclUnhandledCudaError;
    hipMemcpy(d.dTbs, hdr.data(), hdr.size() * sizeof(DevTbHeader), hipMemcpyHostToDevice);
    hipMemcpy(d.dBlob, blob.data(), blob.size(), hipMemcpyHostToDevice);
    comm->devAlgos.push_back(d);
  }
  return ringUpload(comm);
}

}  // namespace msccl

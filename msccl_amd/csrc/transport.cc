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
  comm->buffSizes[kProtoLL] = (int)envInt("NCCL_LL_BUFFSIZE", 8 * 512 * kFifoSteps * 16);
  comm->buffSizes[kProtoLL128] = (int)envInt("NCCL_LL128_BUFFSIZE", 120 * 640 * kFifoSteps * 8);
  comm->buffSizes[kProtoSimple] = (int)envInt("NCCL_BUFFSIZE", 1 << 22);
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
  comm->sendKeys.clear();
  comm->recvKeys.clear();
  comm->sendProtoMask.clear();
  comm->recvProtoMask.clear();
  for (auto& kv : sends) { comm->sendKeys.push_back(kv.first); comm->sendProtoMask.push_back(kv.second); }
  for (auto& kv : recvs) { comm->recvKeys.push_back(kv.first); comm->recvProtoMask.push_back(kv.second); }

  const int S = comm->maxSplit;
  const int64_t llBytes = (int64_t)alignUp((size_t)kFifoSteps * comm->llSlotLines * 16, kFifoAlign);
  const int64_t simpleBytes = (int64_t)alignUp((size_t)kFifoSteps * comm->simpleSlotBytes, kFifoAlign);
  comm->table.assign((size_t)kMaxChannels * n, PeerOffsets{-1, -1, -1, -1, llBytes, simpleBytes, (int64_t)kWordStride, 0});
  size_t off = 0;
  for (auto& k : comm->sendKeys) { comm->table[(size_t)k.chan * n + k.peer].sendHead = (int64_t)off; off += kWordStride * S; }
  for (auto& k : comm->recvKeys) { comm->table[(size_t)k.chan * n + k.peer].recvTail = (int64_t)off; off += kWordStride * S; }
  off = alignUp(off, kFifoAlign);
  for (size_t i = 0; i < comm->recvKeys.size(); i++) {
    auto& k = comm->recvKeys[i];
    PeerOffsets& po = comm->table[(size_t)k.chan * n + k.peer];
    // LL128 schedules run on the LL FIFO format in this build
    if (comm->recvProtoMask[i] & ((1u << kProtoLL) | (1u << kProtoLL128))) {
      po.recvLL = (int64_t)off;
      off += (size_t)llBytes * S;
    }
    if (comm->recvProtoMask[i] & (1u << kProtoSimple)) {
      po.recvSimple = (int64_t)off;
      off += (size_t)simpleBytes * S;
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

// Pack every algorithm's per-tb programs and upload them (replaces the 29 MB
// mscclDevCommInfo copy of devCommSetup, init.cc:300-304).
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
  return ncclSuccess;
}

}  // namespace msccl

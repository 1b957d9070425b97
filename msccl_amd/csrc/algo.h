// MSCCL algorithm (schedule) data model — host side.
//
// Restates the schedule content of the reference's include/msccl.h:6-166
// (mscclTransfer, mscclThreadBlock, mscclAlgorithm, limits and op codes) in a
// form sized for what this runtime actually ships to the device: the host keeps
// the full per-tb program, the device gets a packed blob (see device/devcomm.h).
#pragma once
#include <stdint.h>
#include <string>
#include <vector>

namespace msccl {

// Limits — identical values to include/msccl.h:6-14 and devcomm.h:33,53-55.
constexpr int kMaxSteps = 256;              // MSCCL_MAX_NUM_STEPS
constexpr int kMaxTbPerChannel = 32;        // MSCCL_MAX_NUM_THREAD_BLOCKS_PER_CHANNEL
constexpr int kMaxTb = 216;                 // MSCCL_MAX_NUM_THREAD_BLOCKS
constexpr int kMaxAlgos = 4;                // MSCCL_MAX_NUM_ALGOS
constexpr int kMaxCount = 72;               // MSCCL_MAX_COUNT
constexpr int kMaxReduceFusion = 16;        // MSCCL_MAX_REDUCE_FUSION
constexpr int kMaxChannels = 32;            // MAXCHANNELS
constexpr int kSteps = 8;                   // NCCL_STEPS
constexpr int kSliceSteps = kSteps / 4;     // MSCCL_SLICESTEPS
constexpr int kChunkSteps = kSteps / 2;     // MSCCL_CHUNKSTEPS
constexpr int kRefWarp = 32;                // reference WARP_SIZE (used only in the chunk math)
constexpr int kMaxIter = 65536;             // MSCCL_MAX_ITER (msccl_interpreter.h:10)
// Ring fallback (enqueue.cc:461-476): channels kRingChanBase.. of the connection table carry
// one ring (send to rank+1, receive from rank-1) each; XML channels are 0..32.
constexpr int kRingChannels = 32;  // as many as the reference's MAXCHANNELS
constexpr int kRingChanBase = 40;
constexpr int kTableChannels = kRingChanBase + kRingChannels;

// Buffer ids (msccl.h:19-21)
enum BufId : uint8_t { kInput = 0, kOutput = 1, kScratch = 2 };

// Transfer types (msccl.h:23-31)
enum OpType : uint8_t {
  kSend = 0, kRecv = 1, kRecvCopySend = 2, kRecvReduceSend = 3, kRecvReduceCopy = 4,
  kRecvReduceCopySend = 5, kLocalCopy = 6, kReduce = 7, kResAdd = 8,
  kCopySend = 9,  // ring AllGather out of place (directCopySend, all_gather.h:59); never from XML
  // `s` fused with the `rrc` that follows it (same source chunks, same peer): the device image of
  // a thread block whose exchange both ends run as one pass (transport.cc: fusableTbs); never
  // from XML
  kSendRecvReduceCopy = 10,
  // `s` fused with the `cpy` of the same source chunks that follows it: one pass that sends the
  // source and copies it (the ring's copy-send); never from XML
  kSendCopy = 11,
  // the flat tree's fold (transport.cc: ringUpload): receive every peer's input over the recv
  // connections of thread blocks 1..n-1 and fold all n inputs, in the order of the reduction
  // table (thread block per position, -1 = this rank's input), into the output; never from XML
  kFoldRecv = 12
};

// Device reduction ops (ncclDevRedOp_t, devcomm.h): Sum, Prod, Max, Min, PreMulSum, SumPostDiv
enum DevRedOp : int { kDevSum = 0, kDevProd = 1, kDevMax = 2, kDevMin = 3, kDevPreMulSum = 4, kDevSumPostDiv = 5 };

// Protocol ids (devcomm.h:27-29)
enum Proto : int { kProtoLL = 0, kProtoLL128 = 1, kProtoSimple = 2, kNumProtos = 3 };

// ncclFunc_t (devcomm.h:16)
enum Coll : int {
  kBroadcast = 0, kReduceColl = 1, kAllGather = 2, kReduceScatter = 3, kAllReduce = 4,
  kAllToAll = 5, kCustom = 6, kSendRecv = 7, kSendColl = 8, kRecvColl = 9
};

struct Transfer {
  int16_t srcoff = 0, dstoff = 0;
  uint8_t srcbuf = 0, dstbuf = 0;
  int16_t depPtr = 0, numDeps = 0;     // into ThreadBlock::depBid/depStep
  int8_t hasDep = 0;
  int16_t numReds = 0, redPtr = 0;     // into ThreadBlock::redSrcOff
  uint8_t type = 0, count = 0;
};

struct ThreadBlock {
  int16_t sendpeer = -1, recvpeer = -1;
  uint16_t nsteps = 0;
  int8_t channel = 0;
  bool exists = false;
  // dependentBid is int8_t in the reference (msccl.h:57): a dependency on a
  // tb id >= 128 overflows there.  Kept wide here; the loader records it.
  std::vector<int16_t> depBid, depStep, redSrcOff;
  std::vector<Transfer> transfers;
};

struct Algorithm {
  std::string name;
  bool valid = false;
  int coll = kAllReduce;
  int inPlace = 0;
  int ngpus = 0;
  int nchunksPerLoop = 0;
  int proto = kProtoSimple;
  int64_t minBytes = 0, maxBytes = 0;
  int nChannels = 0;       // XML nchannels attribute
  int nBlocks = 0;
  int nThreads = 0;        // XML nthreads attribute (0 = unset)
  int nScratchChunks = 0;
  int nInputChunks = 0, nOutputChunks = 0;
  std::vector<ThreadBlock> tbs;   // size nBlocks
  std::string path;
};

// Registration from MSCCL_CONFIG (msccl.h:140-145)
struct Registration {
  int algoIndex;
  int64_t minBytes, maxBytes;  // maxBytes == -1 means unbounded
  int proto;
};

// Loader entry points (xml.cc).  Return ncclResult_t codes (0 = success).
int loadAlgoFromXml(const char* path, Algorithm* algo, int maxNChannels, int rank, int nRanks);
int loadAlgosFromXmlFiles(const char* list, std::vector<Algorithm>* algos, int maxNChannels, int rank, int nRanks);
int loadAlgosFromConfig(const char* path, std::vector<Algorithm>* algos, std::vector<Registration>* regs,
                        int maxNChannels, int rank, int nRanks);

// JSON dump of the loaded program (used by tests to compare with the oracle).
std::string algoToJson(const Algorithm& a);

}  // namespace msccl

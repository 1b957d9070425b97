// Lowering of one-hop MSCCL AllReduce schedules to the flat fold kernel (lower.cc).
#pragma once
#include <string>
#include <vector>

#include "algo.h"

namespace msccl {

// byRank[r]: the schedule as loaded for rank r (every rank of the communicator).  ok: on every
// rank r every result chunk c is a left fold over all ranks of their chunk c,
// x_{o(0)}[c] (+) x_{o(1)}[c] (+) ... (+) x_{o(n-1)}[c], under the LL protocol's semantics, so the
// flat fold kernel with those orders computes the schedule's values; why: the reason it is not.
// The chunks fall into classes of identical orders on every rank (a one-shot: one class; the
// two-phase all-pairs: one per chunk owner, who folds its own chunk first):
//   chunkClass[c]       the class of chunk c (classes numbered by their first chunk);
//   order[k][r]         the fold order (ranks) of class k on rank r.
//
// twoPhase: besides, every rank's result chunk c is one and the same expression (every rank holds
// the bits its owner computed), and every rank owns C / n chunks; owner[c] is the rank whose
// transfer computed chunk c's final fold (the msccl-tools two-phase all-pairs: the rank whose
// `re` folds it, before its `s` hands it to the peers).  The two-phase fold kernel then runs the
// schedule's dataflow without its scratch round trip: every rank sends chunk c of its input to
// owner[c]; the owner folds the n copies straight from the FIFO lines in order[class(c)][owner]
// and sends the result to every peer (interpreter.h: runTwoPhase).
struct FoldLowering {
  bool ok = false;
  std::string why;
  std::vector<int> chunkClass;
  std::vector<std::vector<std::vector<int>>> order;
  bool twoPhase = false;
  std::string whyNotTwoPhase;
  std::vector<int> owner;
};
FoldLowering analyzeFoldLowering(const std::vector<Algorithm>& byRank);

// The direct form of a Simple schedule (the reference's P2P direct mode, prims_simple.h:75-128,
// 500-560: within one process a sender writes straight into the receiver's buffer).  When every
// rank of a communicator sits in one fused launch (ncclCommInitAll on one GPU, one group call),
// every rank's buffers are addressable from the launch and ready at its start, so the schedule's
// values need no FIFO at all:
//   AllGather (out of place): ok when every output chunk is its rank's input chunk (the
//     AllGather's definition): each rank writes its input into every rank's output once;
//   ReduceScatter (out of place): ok when rank r's output chunk c is a left fold of every rank's
//     input chunk r C / n + c; rank r reads every rank's block and folds it in order[k][r];
//   AllReduce: ok when chunk c is one left fold of every rank's chunk c, the same value on every
//     rank; rank r folds its share of the packs in order[k][.] and writes it to every rank.
// Simple's semantics: `re` folds (s_0 (+) s_1 ...) (+) d (prims_simple.h:258-263; calls whose every
// transfer moves at least nthreads elements, plan.cc: the direct plan's guard), rrs / rrc
// fn(local, peer).  chunkClass is per output chunk (RS: C / n of them).
struct DirectLowering {
  bool ok = false;
  std::string why;
  int coll = -1;
  std::vector<int> chunkClass;
  std::vector<std::vector<std::vector<int>>> order;
};
DirectLowering analyzeDirectLowering(const std::vector<Algorithm>& byRank);
// the file loaded for each of nRanks ranks, then analyzeDirectLowering (cached like lowerScheduleFile)
DirectLowering directScheduleFile(const std::string& path, int nRanks);
// The schedule file at `path` loaded for each of nRanks ranks, then analyzeFoldLowering; cached
// per process by (file text, nRanks), so the co-resident communicators of one process (each
// rank loads it for every rank) parse and analyse a file once.  A file that does not load for
// some rank is not lowered.
FoldLowering lowerScheduleFile(const std::string& path, int nRanks);
// false when this rank records the schedule's own primitives (MSCCL_AMD_NPKIT, MSCCL_AMD_TRACE=1):
// it then offers no lowering at init, and every rank keeps the interpreter
bool lowerOffered();

}  // namespace msccl

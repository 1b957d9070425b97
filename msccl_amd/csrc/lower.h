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
// The schedule file at `path` loaded for each of nRanks ranks, then analyzeFoldLowering; cached
// per process by (file text, nRanks), so the co-resident communicators of one process (each
// rank loads it for every rank) parse and analyse a file once.  A file that does not load for
// some rank is not lowered.
FoldLowering lowerScheduleFile(const std::string& path, int nRanks);
// false when this rank records the schedule's own primitives (MSCCL_AMD_NPKIT, MSCCL_AMD_TRACE=1):
// it then offers no lowering at init, and every rank keeps the interpreter
bool lowerOffered();

}  // namespace msccl

// Lowering of one-hop MSCCL AllReduce schedules to the flat fold kernel (lower.cc).
#pragma once
#include <string>
#include <vector>

#include "algo.h"

namespace msccl {

// byRank[r]: the schedule as loaded for rank r (every rank of the communicator).  ok: on every
// rank r every result chunk c is x_{order[r][0]}[c] (+) x_{order[r][1]}[c] (+) ... (+)
// x_{order[r][n-1]}[c] (a left fold over all ranks, one order per rank) under the LL protocol's
// semantics, so the flat fold kernel with that order computes the schedule's values; why: the
// reason it is not.
struct FoldLowering {
  bool ok = false;
  std::string why;
  std::vector<std::vector<int>> order;
};
FoldLowering analyzeFoldLowering(const std::vector<Algorithm>& byRank);

}  // namespace msccl

// Group semantics (reference group.cc:17-408): thread-local nesting depth; collectives issued
// inside a group are collected and launched at the outermost ncclGroupEnd, ranks that share a
// GPU are fused into one kernel launch; ncclCommInitRank inside a group runs in parallel threads.
#pragma once
#include <functional>
#include <vector>

#include "../../include/nccl.h"

namespace msccl {

struct CollOp {
  ncclComm* comm;
  int coll;
  const void* sendbuff;
  void* recvbuff;
  size_t count;
  ncclDataType_t dtype;
  ncclRedOp_t op;
  hipStream_t stream;
  int customAlgo;
  // device reduction (hostToDevRedOp, enqueue.cc:1388-1454): 0..3 Sum/Prod/Max/Min,
  // 4 PreMulSum (scale bits or scale address in redArg), 5 SumPostDiv (divisor in redArg)
  int devOp = 0;
  uint64_t redArg = 0;
  int redArgIsPtr = 0;
};

bool groupActive();
void groupAddInit(std::function<ncclResult_t()> fn, ncclComm* comm);
void groupAddOp(const CollOp& op);
ncclResult_t executeOps(std::vector<CollOp>& ops);  // enqueue.cc

}  // namespace msccl

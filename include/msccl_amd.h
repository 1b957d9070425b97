/*
 * msccl-amd — introspection C-ABI used by the tests and the benchmark.
 *
 * These entry points have no counterpart in the reference's public header; they expose the
 * host-side pieces of the MSCCL path (XML loader, selection + chunk math, bootstrap) so the
 * parity tests can compare them with the CPU oracle without a GPU.
 */
#ifndef MSCCL_AMD_H_
#define MSCCL_AMD_H_

#include <stddef.h>
#include "nccl.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Load one MSCCL XML file as rank `rank` of `nranks` (graph/topo.cc:759-1193) and write the
 * resulting program as JSON into out[0..outLen).  Returns the ncclResult_t of the load. */
int mscclAmdAlgoJson(const char* xmlPath, int rank, int nranks, char* out, size_t outLen);

/* The thread blocks of that program whose first FIFO transfers are an `s` then an `rrc` of the same
 * source chunks with one peer: the exchanges this rank offers to run fused (init fuses one only
 * when the peer's thread block on the connection offers it too).  JSON {"fusable":[[tb, index,
 * channel, peer], ...]}.  No GPU needed. */
int mscclAmdFusableJson(const char* xmlPath, int rank, int nranks, char* out, size_t outLen);

/* Whether the AllReduce schedule of one MSCCL XML file, loaded for every rank of `nranks`, runs as
 * the one-hop fold (msccl_amd/csrc/lower.cc: every result chunk of every rank is a left fold of all
 * ranks' same chunk; chunks fall into classes of equal orders).  JSON {"ok":1,"classes":[[[ranks of
 * rank 0's fold], ... per rank], ... per class],"chunkClass":[class of chunk 0, ...]} or
 * {"ok":0,"why":"..."}.  With "ok":1 also "twoPhase":1 and every chunk's "owner" when every rank
 * holds the same fold of every chunk and the ranks own equal shares (the two-phase fold of large
 * calls), else "twoPhase":0 and "whyNotTwoPhase".  No GPU needed. */
int mscclAmdLowerJson(const char* xmlPath, int nranks, char* out, size_t outLen);

/* Whether a Simple AllReduce / ReduceScatter / AllGather schedule has the direct form (lower.h:
 * DirectLowering; run when every rank of a communicator is in one launch).  JSON {"ok":1,"coll":c,
 * "classes":[[[rank r's fold order], ... per rank], ... per class],"chunkClass":[...]} (the
 * AllGather: no classes) or {"ok":0,"coll":c,"why":"..."}.  No GPU needed. */
int mscclAmdDirectJson(const char* xmlPath, int nranks, char* out, size_t outLen);

/* Select among the ':'-separated XML files (tuning.cc:344-382) and compute the schedule's chunk
 * plan (enqueue.cc:591-734), the reference's computeColl field by field, from the environment
 * alone: not init's decisions (lowering to the fold, the local Simple FIFO; see
 * mscclAmdLaunchPlanJson).  coll uses ncclFunc_t numbering (AllGather=2, ReduceScatter=3,
 * AllReduce=4).  Writes JSON {"algo":i,...} or {"algo":-1}.  No GPU needed. */
int mscclAmdPlanJson(const char* xmlFiles, int rank, int nranks, int coll, size_t count, int dtype,
                     int redop, int inPlace, char* out, size_t outLen);

/* What a communicator of `nranks` ranks launches for one call, with init's decisions: all ranks
 * on one GPU (oneGpu = 1) or spread over GPUs (oneGpu = 0: every rank has peers over xGMI).  The
 * same planning function as the communicator's (plan.cc: planCall) on the same inputs: the
 * schedules, the one-hop lowering and its size limit (co-resident: measured; across GPUs: the
 * link model), the Simple FIFO size, the fallback, the pair kernel (a one-pass
 * call of a schedule in pair form on every rank).  JSON {"kernel": "fold" | "pair" | "twophase" |
 * "interpreter" | "ring" | "tree", "kernelExact", "algo", "proto", "lowered", "nBytes",
 * "lowerMaxBytes", "simpleBuffBytes", "remote", "pairForm", "classes": [fold orders per
 * algorithm, 0 = not lowered]}.  "kernelExact" is 0 when the answer for a multi-iteration
 * pair-form call rests on the default FIFO and split (a non-default NCCL_LL_BUFFSIZE or a forced
 * MSCCL_AMD_SPLIT: the communicator's one-pass bound follows its agreed split and FIFO geometry,
 * which this call does not model).  The direct form (a launch holding every rank of a
 * communicator) is not reported here: see mscclAmdDirectJson.  No GPU needed. */
int mscclAmdLaunchPlanJson(const char* xmlFiles, int rank, int nranks, int oneGpu, int coll, size_t count,
                           int dtype, int redop, int inPlace, char* out, size_t outLen);

/* Communicator summary as JSON (algorithms, connections, scratch, FIFO geometry). */
int mscclAmdCommInfo(ncclComm_t comm, char* out, size_t outLen);

/* Bootstrap only (no GPU): rank 0 passes the id from ncclGetUniqueId; every rank contributes
 * `bytes` bytes and receives nranks*bytes in `out`. */
int mscclAmdBootstrapAllgather(const ncclUniqueId* id, int rank, int nranks, const void* mine, size_t bytes,
                               void* out);

/* Number of thread blocks a launch of algorithm `algoIndex` uses on this rank. */
int mscclAmdAlgoBlocks(ncclComm_t comm, int algoIndex);

/* Host-only build check (no GPU needed): the name of the first element type whose kernel object
   was compiled with another RankWork layout than this library's host code ("float32", ...), or
   NULL when every object agrees.  Communicator setup refuses such a library (ncclInternalError);
   tools/varbuild.sh runs this right after linking a measurement variant, before any GPU run. */
const char* mscclAmdKernelLayoutMismatch(void);

/* Device event trace (NPKit-style, the reference's src/include/npkit/): enabled per communicator
 * with MSCCL_AMD_TRACE=1 at init.  Each workgroup slot (tb * maxSplit + sub) records up to
 * MSCCL_AMD_TRACE_EVENTS 16-byte events of its most recent launch:
 *   struct { uint64_t ts;  // s_memrealtime, 100 MHz
 *            uint16_t type; uint16_t step; uint32_t arg; }
 * Event 0 of a slot is a header {ts = launch start, type = 0xFFFF, step = events, arg = epoch}.
 * Copies the whole buffer (slots x events x 16 B) into out; *slots and *events receive the
 * geometry.  Synchronises the device.  ncclInvalidUsage when tracing is off. */
int mscclAmdTraceRead(ncclComm_t comm, void* out, size_t outBytes, int* slots, int* events);

/* 16-B line atomicity probe: the gate for LL128 towards another GPU (the
 * reference enables LL128 only where line atomicity holds, tuning.cc:210-214).  Writers on
 * `writerDev` store nLines 16-B lines {payload(k), payload(k), payload(k), k} for k = 1..iters
 * into uncached memory of `readerDev` (the FIFO memory) while readers there poll them with 16-B
 * loads for at most `seconds`.  out[0] = lines observed with a flag, out[1] = observed lines whose
 * payload does not match their flag (torn), out[2] = lines that reached k = iters. */
int mscclAmdLineTearProbe(int writerDev, int readerDev, int nLines, int iters, double seconds,
                          unsigned long long* out);

/* Read one NAME=VALUE parameter file into the environment without overwriting variables that are
 * already set: the reference's setEnvFile (misc/param.cc:25-49), which its initEnv applies to
 * ~/.nccl.conf and then /etc/nccl.conf before the first parameter read (this library does the
 * same on its first entry).  Returns 0, or ncclSystemError when the file cannot be opened. */
int mscclAmdSetEnvFile(const char* path);

#ifdef __cplusplus
}
#endif
#endif

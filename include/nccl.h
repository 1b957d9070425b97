/*
 * msccl-amd — public C-ABI (drop-in for the reference's src/nccl.h.in).
 *
 * Every declaration below replaces the entry point of the same name in the
 * reference header /root/reference/src/nccl.h.in (line numbers cited per
 * symbol).  Enum values, argument order and the meaning of every argument are
 * identical, so an application (nccl-tests, PyTorch ProcessGroupNCCL) that was
 * compiled against the reference header links against libmsccl_amd.so
 * unchanged.  The only type substitution is cudaStream_t -> hipStream_t (both
 * are opaque pointers to a runtime stream object).
 *
 * Implemented natively for AMD Instinct MI355X (gfx950): the MSCCL schedule
 * interpreter and its LL / Simple primitives are hand-written HIP kernels and
 * peers are reached over xGMI (peer pointers / hipIpc).
 */
#ifndef MSCCL_AMD_NCCL_H_
#define MSCCL_AMD_NCCL_H_

#include <hip/hip_runtime_api.h>
#include <stddef.h>

#define NCCL_MAJOR 2
#define NCCL_MINOR 12
#define NCCL_PATCH 12
#define MSCCL_VERSION 0.7.4
#define NCCL_SUFFIX "msccl-amd"

#define NCCL_VERSION_CODE 21212
#define NCCL_VERSION(X,Y,Z) (((X) <= 2 && (Y) <= 8) ? (X) * 1000 + (Y) * 100 + (Z) : (X) * 10000 + (Y) * 100 + (Z))

#ifdef __cplusplus
extern "C" {
#endif

/* Opaque handle to communicator (nccl.h.in:30) */
typedef struct ncclComm* ncclComm_t;

#define NCCL_UNIQUE_ID_BYTES 128
typedef struct { char internal[NCCL_UNIQUE_ID_BYTES]; } ncclUniqueId;   /* nccl.h.in:32-33 */

/* Error type (nccl.h.in:36-42) */
typedef enum { ncclSuccess                 =  0,
               ncclUnhandledCudaError      =  1,
               ncclSystemError             =  2,
               ncclInternalError           =  3,
               ncclInvalidArgument         =  4,
               ncclInvalidUsage            =  5,
               ncclNumResults              =  6 } ncclResult_t;

/* nccl.h.in:48 — returns NCCL_VERSION_CODE */
ncclResult_t  ncclGetVersion(int *version);

/* nccl.h.in:54 — 128-byte opaque id; carries the bootstrap root address */
ncclResult_t  ncclGetUniqueId(ncclUniqueId* uniqueId);

/* nccl.h.in:63 — one rank per process (or thread), rendezvous through uniqueId */
ncclResult_t  ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId commId, int rank);

/* nccl.h.in:72 — single process, ndev ranks; devlist may repeat a device
 * (co-resident ranks on one MI355X, driven by one fused launch per group) */
ncclResult_t  ncclCommInitAll(ncclComm_t* comm, int ndev, const int* devlist);

/* nccl.h.in:77,82 */
ncclResult_t  ncclCommDestroy(ncclComm_t comm);
ncclResult_t  ncclCommAbort(ncclComm_t comm);

/* nccl.h.in:86,90,94,98,102 */
const char*   ncclGetErrorString(ncclResult_t result);
ncclResult_t  ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t *asyncError);
ncclResult_t  ncclCommCount(const ncclComm_t comm, int* count);
ncclResult_t  ncclCommCuDevice(const ncclComm_t comm, int* device);
ncclResult_t  ncclCommUserRank(const ncclComm_t comm, int* rank);

/* Reduction operation selector (nccl.h.in:106-121) */
typedef enum { ncclNumOps_dummy = 5 } ncclRedOp_dummy_t;
typedef enum { ncclSum        = 0,
               ncclProd       = 1,
               ncclMax        = 2,
               ncclMin        = 3,
               ncclAvg        = 4,
               ncclNumOps     = 5,
               ncclMaxRedOp   = 0x7fffffff>>(32-8*sizeof(ncclRedOp_dummy_t))
             } ncclRedOp_t;

/* Data types (nccl.h.in:125-140); bf16 is always present on gfx950 */
typedef enum { ncclInt8       = 0, ncclChar       = 0,
               ncclUint8      = 1,
               ncclInt32      = 2, ncclInt        = 2,
               ncclUint32     = 3,
               ncclInt64      = 4,
               ncclUint64     = 5,
               ncclFloat16    = 6, ncclHalf       = 6,
               ncclFloat32    = 7, ncclFloat      = 7,
               ncclFloat64    = 8, ncclDouble     = 8,
               ncclBfloat16   = 9,
               ncclNumTypes   = 10
} ncclDataType_t;

/* nccl.h.in:143-151 */
typedef enum {
  ncclScalarDevice = 0,
  ncclScalarHostImmediate = 1
} ncclScalarResidence_t;

/* nccl.h.in:153-174.  Creates a PreMulSum user op: every input is multiplied by *scalar before
 * the sum (the scalar is read at call time from host memory, ncclScalarHostImmediate, or at
 * kernel time from device memory, ncclScalarDevice).  Like ncclAvg, such ops are never
 * MSCCL-eligible (tuning.cc:345): they run on the ring fallback. */
ncclResult_t  ncclRedOpCreatePreMulSum(ncclRedOp_t *op, void *scalar, ncclDataType_t datatype, ncclScalarResidence_t residence, ncclComm_t comm);
ncclResult_t  ncclRedOpDestroy(ncclRedOp_t op, ncclComm_t comm);

/* Collectives (nccl.h.in:241-277).  Return after enqueue on `stream`.
 * AllReduce in-place iff sendbuff == recvbuff;
 * ReduceScatter in-place iff recvbuff == sendbuff + rank*recvcount*typesize;
 * AllGather in-place iff sendbuff == recvbuff + rank*sendcount*typesize. */
ncclResult_t  ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count,
    ncclDataType_t datatype, ncclRedOp_t op, ncclComm_t comm, hipStream_t stream);
ncclResult_t  ncclReduceScatter(const void* sendbuff, void* recvbuff,
    size_t recvcount, ncclDataType_t datatype, ncclRedOp_t op, ncclComm_t comm,
    hipStream_t stream);
ncclResult_t  ncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount,
    ncclDataType_t datatype, ncclComm_t comm, hipStream_t stream);

/* nccl.h.in:290 — MSCCL-only AllToAll (an alltoall XML must be loaded). */
ncclResult_t  ncclAllToAll(const void* sendbuff, void* recvbuff, size_t sendcount,
    ncclDataType_t datatype, ncclComm_t comm, hipStream_t stream);

/* nccl.h.in:301 — runs XML algorithm number mscclAlgorithmIndex (coll="custom"). */
ncclResult_t  ncclCustomCollective(const void* sendbuff, void* recvbuff, size_t count,
    ncclDataType_t datatype, int mscclAlgorithmIndex, ncclComm_t comm, hipStream_t stream);

/* Group semantics (nccl.h.in:369-380) */
ncclResult_t  ncclGroupStart();
ncclResult_t  ncclGroupEnd();

/* nccl.h.in:382 */
const char*  ncclGetLastError(ncclComm_t comm);

#ifdef __cplusplus
} // end extern "C"
#endif

#endif // MSCCL_AMD_NCCL_H_

/*
 * msccl-amd — NPKit-compatible event log of the interpreter kernel.
 *
 * Enabled per communicator with MSCCL_AMD_NPKIT=1 at init (the reference enables it at build
 * time, makefiles/common.mk:95-97 ENABLE_NPKIT).  Every thread block of every launch appends
 * 16-byte events to its own buffer (buffer = thread block index, as the reference's
 * NPKIT_GPU_SYNC_TIME(bid, tid); the tree fallback's two workgroups of channel c are buffers
 * 2c / 2c+1 as NPKIT_GPU_SYNC_TIME_TREE_SPLIT).  Buffers keep events across launches, up to
 * MSCCL_AMD_NPKIT_EVENTS per buffer (default 65536, NpKit::kMaxNumGpuEventsPerBuffer).
 *
 * Dump (ncclCommDestroy / ncclCommAbort, or mscclAmdNpkitDump) into $NPKIT_DUMP_DIR (default
 * /tmp/), the file set of the reference's NpKit::Dump (src/misc/npkit.cc:64-127):
 *   gpu_events_rank_<r>_buf_<b>       b = 0..511, the events of buffer b (may be empty)
 *   cpu_events_rank_<r>_channel_<c>   c = 0..31; empty: the reference records CPU events only in
 *                                     its network proxy (transport/net.cc), which the xGMI
 *                                     path has no counterpart of
 *   cpu_clock_period_num_rank_<r>     "1"           CPU timestamps are nanoseconds
 *   cpu_clock_period_den_rank_<r>     "1000000000"
 *   gpu_clock_rate_rank_<r>           GPU timestamp rate in kHz (s_memrealtime: 100000)
 * so the reference's tools/npkit_trace_generator.py reads it unchanged; msccl_amd/npkit.py
 * converts it to the same Chrome trace.
 *
 * Event layout (npkit_struct.h:8-17, little endian): byte 0 type, bytes 1-4 size, bytes 5-7
 * rsvd, bytes 8-15 timestamp.  Each launch of a thread block starts with TIME_SYNC_CPU
 * (timestamp = host system_clock ns of the launch start, from the GPU clock and a per-
 * communicator calibration instead of the reference's host-mapped counter thread) and
 * TIME_SYNC_GPU (the GPU clock); then DEP_CHECK_ENTRY/EXIT (size = dependencies) around each
 * dependency wait and <primitive>_ENTRY/EXIT (size = bytes of the call) around each primitive
 * call, as msccl_interpreter.h:88-201 and prims_ll.h:455-536 place them.
 */
#ifndef MSCCL_AMD_NPKIT_H_
#define MSCCL_AMD_NPKIT_H_

#include <stddef.h>
#include "nccl.h"

/* Event ids: the values of the reference's src/include/npkit/npkit_event.h (same numbers, so
 * either trace generator maps them to the same names). */
#define NPKIT_EVENT_INVALID 0x0
#define NPKIT_EVENT_SEND_ENTRY 0x1
#define NPKIT_EVENT_SEND_EXIT 0x2
#define NPKIT_EVENT_SEND_FROM_OUTPUT_ENTRY 0x3
#define NPKIT_EVENT_SEND_FROM_OUTPUT_EXIT 0x4
#define NPKIT_EVENT_DIRECT_SEND_ENTRY 0x5
#define NPKIT_EVENT_DIRECT_SEND_EXIT 0x6
#define NPKIT_EVENT_DIRECT_SEND_FROM_OUTPUT_ENTRY 0x7
#define NPKIT_EVENT_DIRECT_SEND_FROM_OUTPUT_EXIT 0x8
#define NPKIT_EVENT_RECV_ENTRY 0x9
#define NPKIT_EVENT_RECV_EXIT 0xA
#define NPKIT_EVENT_DIRECT_RECV_ENTRY 0xB
#define NPKIT_EVENT_DIRECT_RECV_EXIT 0xC
#define NPKIT_EVENT_REDUCE_ENTRY 0xD
#define NPKIT_EVENT_REDUCE_EXIT 0xE
#define NPKIT_EVENT_LOCAL_COPY_ENTRY 0xF
#define NPKIT_EVENT_LOCAL_COPY_EXIT 0x10
#define NPKIT_EVENT_COPY_SEND_ENTRY 0x11
#define NPKIT_EVENT_COPY_SEND_EXIT 0x12
#define NPKIT_EVENT_DIRECT_COPY_SEND_ENTRY 0x13
#define NPKIT_EVENT_DIRECT_COPY_SEND_EXIT 0x14
#define NPKIT_EVENT_RECV_COPY_SEND_ENTRY 0x15
#define NPKIT_EVENT_RECV_COPY_SEND_EXIT 0x16
#define NPKIT_EVENT_DIRECT_RECV_COPY_SEND_ENTRY 0x17
#define NPKIT_EVENT_DIRECT_RECV_COPY_SEND_EXIT 0x18
#define NPKIT_EVENT_RECV_COPY_DIRECT_SEND_ENTRY 0x19
#define NPKIT_EVENT_RECV_COPY_DIRECT_SEND_EXIT 0x1A
#define NPKIT_EVENT_RECV_REDUCE_COPY_ENTRY 0x1B
#define NPKIT_EVENT_RECV_REDUCE_COPY_EXIT 0x1C
#define NPKIT_EVENT_RECV_REDUCE_SEND_ENTRY 0x1D
#define NPKIT_EVENT_RECV_REDUCE_SEND_EXIT 0x1E
#define NPKIT_EVENT_DIRECT_RECV_REDUCE_SEND_ENTRY 0x1F
#define NPKIT_EVENT_DIRECT_RECV_REDUCE_SEND_EXIT 0x20
#define NPKIT_EVENT_RECV_REDUCE_COPY_SEND_ENTRY 0x21
#define NPKIT_EVENT_RECV_REDUCE_COPY_SEND_EXIT 0x22
#define NPKIT_EVENT_DIRECT_RECV_REDUCE_COPY_SEND_ENTRY 0x23
#define NPKIT_EVENT_DIRECT_RECV_REDUCE_COPY_SEND_EXIT 0x24
#define NPKIT_EVENT_NET_SEND_ENTRY 0x25
#define NPKIT_EVENT_NET_SEND_EXIT 0x26
#define NPKIT_EVENT_NET_RECV_ENTRY 0x27
#define NPKIT_EVENT_NET_RECV_EXIT 0x28
#define NPKIT_EVENT_DEP_CHECK_ENTRY 0x29
#define NPKIT_EVENT_DEP_CHECK_EXIT 0x2A
#define NPKIT_EVENT_TIME_SYNC_GPU 0x2B
#define NPKIT_EVENT_TIME_SYNC_CPU 0x2C

#define MSCCL_AMD_NPKIT_GPU_BUFFERS 512 /* NpKit::kNumGpuEventBuffers */
#define MSCCL_AMD_NPKIT_CPU_BUFFERS 32  /* NpKit::kNumCpuEventBuffers */

#ifdef __cplusplus
extern "C" {
#endif

/* Write the communicator's NPKit dump into `dir` (NULL: $NPKIT_DUMP_DIR, else /tmp/) now;
 * synchronises the device.  ncclInvalidUsage when MSCCL_AMD_NPKIT was off at init. */
int mscclAmdNpkitDump(ncclComm_t comm, const char* dir);

#ifdef __cplusplus
}
#endif
#endif

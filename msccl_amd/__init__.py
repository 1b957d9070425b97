"""msccl_amd — MI355X-native MSCCL collectives runtime (Python host binding).

The product is the C-ABI library ``msccl_amd/libmsccl_amd.so`` (public header
``include/nccl.h``: the reference's ncclAllReduce / ncclReduceScatter / ncclAllGather surface,
src/nccl.h.in).  This module binds it with ctypes for tests, benchmarks and Python users, the
way a framework's FFI would.  There is no Python or CPU fallback: if the shared library is
missing every entry point raises.
"""
from __future__ import annotations

import ctypes
import json
import os
from typing import List, Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
# MSCCL_AMD_LIB points at another build of the library (A/B measurements of two builds on one box)
LIB_PATH = os.environ.get("MSCCL_AMD_LIB") or os.path.join(_HERE, "libmsccl_amd.so")

# trace event layout (include/msccl_amd.h: mscclAmdTraceRead); types: 1 setup, 2 dep-wait done,
# 3 primitive begin (arg = transfer type << 24 | elements), 4 primitive end, 5 end, 0xFFFF header
TRACE_DTYPE = [("ts", "<u8"), ("type", "<u2"), ("step", "<u2"), ("arg", "<u4")]
TRACE_TYPES = {1: "setup", 2: "dep", 3: "begin", 4: "end", 5: "done", 0xFFFF: "header"}

# ncclDataType_t (nccl.h.in:125-140)
INT8, UINT8, INT32, UINT32, INT64, UINT64, FLOAT16, FLOAT32, FLOAT64, BFLOAT16 = range(10)
DTYPE_NAMES = {"int8": INT8, "uint8": UINT8, "int32": INT32, "uint32": UINT32, "int64": INT64,
               "uint64": UINT64, "float16": FLOAT16, "fp16": FLOAT16, "float32": FLOAT32, "fp32": FLOAT32,
               "float64": FLOAT64, "fp64": FLOAT64, "bfloat16": BFLOAT16, "bf16": BFLOAT16}
TYPE_SIZE = {INT8: 1, UINT8: 1, INT32: 4, UINT32: 4, INT64: 8, UINT64: 8, FLOAT16: 2, FLOAT32: 4,
             FLOAT64: 8, BFLOAT16: 2}
# ncclRedOp_t (nccl.h.in:106-121)
SUM, PROD, MAX, MIN, AVG = range(5)
SCALAR_DEVICE, SCALAR_HOST = 0, 1  # ncclScalarResidence_t
# ncclFunc_t (devcomm.h:16)
COLL_ALLGATHER, COLL_REDUCE_SCATTER, COLL_ALLREDUCE, COLL_ALLTOALL, COLL_CUSTOM = 2, 3, 4, 5, 6

_ERRS = {0: "ncclSuccess", 1: "ncclUnhandledCudaError", 2: "ncclSystemError", 3: "ncclInternalError",
         4: "ncclInvalidArgument", 5: "ncclInvalidUsage"}


class NcclError(RuntimeError):
    def __init__(self, code: int, where: str):
        self.code = code
        super().__init__("%s failed: %s (%d) %s" % (where, _ERRS.get(code, "?"), code, last_error()))


class UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


_lib = None


def lib() -> ctypes.CDLL:
    """Load libmsccl_amd.so; raises loudly when it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("msccl_amd: %s is missing — run __graft_entry__.build() (make -C msccl_amd/csrc)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    vp, i, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    L.ncclGetVersion.argtypes = [ctypes.POINTER(i)]
    L.ncclGetUniqueId.argtypes = [ctypes.POINTER(UniqueId)]
    L.ncclCommInitRank.argtypes = [ctypes.POINTER(vp), i, UniqueId, i]
    L.ncclCommInitAll.argtypes = [ctypes.POINTER(vp), i, ctypes.POINTER(i)]
    L.ncclCommDestroy.argtypes = [vp]
    L.ncclCommAbort.argtypes = [vp]
    L.ncclGetErrorString.restype = ctypes.c_char_p
    L.ncclGetErrorString.argtypes = [i]
    L.ncclGetLastError.restype = ctypes.c_char_p
    L.ncclGetLastError.argtypes = [vp]
    L.ncclCommGetAsyncError.argtypes = [vp, ctypes.POINTER(i)]
    L.ncclCommCount.argtypes = [vp, ctypes.POINTER(i)]
    L.ncclCommCuDevice.argtypes = [vp, ctypes.POINTER(i)]
    L.ncclCommUserRank.argtypes = [vp, ctypes.POINTER(i)]
    L.ncclAllReduce.argtypes = [vp, vp, sz, i, i, vp, vp]
    L.ncclReduceScatter.argtypes = [vp, vp, sz, i, i, vp, vp]
    L.ncclAllGather.argtypes = [vp, vp, sz, i, vp, vp]
    L.ncclAllToAll.argtypes = [vp, vp, sz, i, vp, vp]
    L.ncclCustomCollective.argtypes = [vp, vp, sz, i, i, vp, vp]
    L.ncclRedOpCreatePreMulSum.argtypes = [ctypes.POINTER(i), vp, i, i, vp]
    L.ncclRedOpDestroy.argtypes = [i, vp]
    L.ncclGroupStart.argtypes = []
    L.ncclGroupEnd.argtypes = []
    L.mscclAmdAlgoJson.argtypes = [ctypes.c_char_p, i, i, ctypes.c_char_p, sz]
    L.mscclAmdFusableJson.argtypes = [ctypes.c_char_p, i, i, ctypes.c_char_p, sz]
    if hasattr(L, "mscclAmdLowerJson"):  # MSCCL_AMD_LIB may name an older build (A/B runs)
        L.mscclAmdLowerJson.argtypes = [ctypes.c_char_p, i, ctypes.c_char_p, sz]
    if hasattr(L, "mscclAmdDirectJson"):
        L.mscclAmdDirectJson.argtypes = [ctypes.c_char_p, i, ctypes.c_char_p, sz]
    if hasattr(L, "mscclAmdKernelLayoutMismatch"):
        L.mscclAmdKernelLayoutMismatch.argtypes = []
        L.mscclAmdKernelLayoutMismatch.restype = ctypes.c_char_p
    L.mscclAmdPlanJson.argtypes = [ctypes.c_char_p, i, i, i, sz, i, i, i, ctypes.c_char_p, sz]
    if hasattr(L, "mscclAmdLaunchPlanJson"):  # MSCCL_AMD_LIB may name an older build (A/B runs)
        L.mscclAmdLaunchPlanJson.argtypes = [ctypes.c_char_p, i, i, i, i, sz, i, i, i, ctypes.c_char_p, sz]
    L.mscclAmdCommInfo.argtypes = [vp, ctypes.c_char_p, sz]
    L.mscclAmdNpkitDump.argtypes = [vp, ctypes.c_char_p]
    L.mscclAmdBootstrapAllgather.argtypes = [ctypes.POINTER(UniqueId), i, i, vp, sz, vp]
    L.mscclAmdAlgoBlocks.argtypes = [vp, i]
    L.mscclAmdTraceRead.argtypes = [vp, vp, sz, ctypes.POINTER(i), ctypes.POINTER(i)]
    if hasattr(L, "mscclAmdLineTearProbe"):  # MSCCL_AMD_LIB may name an older build (A/B runs)
        L.mscclAmdLineTearProbe.argtypes = [i, i, i, i, ctypes.c_double, ctypes.POINTER(ctypes.c_ulonglong)]
    _lib = L
    return L


def last_error() -> str:
    try:
        s = lib().ncclGetLastError(None)
        return s.decode() if s else ""
    except Exception:  # noqa: BLE001
        return ""


def _check(code: int, where: str) -> None:
    if code != 0:
        raise NcclError(code, where)


def version() -> int:
    v = ctypes.c_int()
    _check(lib().ncclGetVersion(ctypes.byref(v)), "ncclGetVersion")
    return v.value


def get_unique_id() -> bytes:
    uid = UniqueId()
    _check(lib().ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
    return ctypes.string_at(ctypes.addressof(uid), 128)  # .internal would stop at the first NUL


def _uid(b: bytes) -> UniqueId:
    if len(b) != 128:
        raise ValueError("ncclUniqueId must be 128 bytes")
    u = UniqueId()
    ctypes.memmove(ctypes.addressof(u), b, 128)
    return u


def algo_json(xml_path: str, rank: int, nranks: int) -> dict:
    """The product loader's program for one rank (graph/topo.cc:759-1193)."""
    buf = ctypes.create_string_buffer(1 << 24)
    _check(lib().mscclAmdAlgoJson(xml_path.encode(), rank, nranks, buf, len(buf)), "mscclAmdAlgoJson")
    return json.loads(buf.value.decode())


def fusable_json(xml_path: str, rank: int, nranks: int, key: str = "fusable") -> list:
    """The exchanges one rank of a schedule offers to run fused (transport.cc: fusableTbs):
    [[tb, index of its s, channel, peer], ...]; key "sendcopy": the s + cpy pairs it runs as one
    copy-send pass (transport.cc: sendCopyFusable), [[tb, index of the s], ...]."""
    buf = ctypes.create_string_buffer(1 << 20)
    _check(lib().mscclAmdFusableJson(xml_path.encode(), rank, nranks, buf, len(buf)), "mscclAmdFusableJson")
    return json.loads(buf.value.decode())[key]


def lower_json(xml_path: str, nranks: int) -> dict:
    """Whether the AllReduce schedule runs as the one-hop fold kernel (msccl_amd/csrc/lower.cc):
    {"ok": 1, "classes": [[fold order of rank 0, ...] per class of chunks], "chunkClass": [class of
    each chunk]} or {"ok": 0, "why": reason}."""
    buf = ctypes.create_string_buffer(1 << 16)
    _check(lib().mscclAmdLowerJson(xml_path.encode(), nranks, buf, len(buf)), "mscclAmdLowerJson")
    return json.loads(buf.value.decode())


def direct_json(xml_path: str, nranks: int) -> dict:
    """Whether a Simple AllReduce / ReduceScatter / AllGather schedule has the direct form (lower.h:
    DirectLowering; it runs when every rank of a communicator is in one launch): {"ok": 1, "coll": c,
    "classes": [[fold order of each rank] per class], "chunkClass": [...]} or {"ok": 0, "why": ...}."""
    buf = ctypes.create_string_buffer(1 << 16)
    _check(lib().mscclAmdDirectJson(xml_path.encode(), nranks, buf, len(buf)), "mscclAmdDirectJson")
    return json.loads(buf.value.decode())


def line_tear_probe(writer_dev: int, reader_dev: int, lines: int = 1 << 16, iters: int = 2000,
                    seconds: float = 5.0) -> dict:
    """mscclAmdLineTearProbe (include/msccl_amd.h): 16-B lines written from one device into another
    device's uncached memory while that device polls them; counts lines seen torn."""
    out = (ctypes.c_ulonglong * 3)()
    _check(lib().mscclAmdLineTearProbe(writer_dev, reader_dev, lines, iters, seconds, out), "mscclAmdLineTearProbe")
    return {"seen": out[0], "torn": out[1], "done": out[2], "lines": lines, "iters": iters}


def try_algo_json(xml_path: str, rank: int, nranks: int):
    buf = ctypes.create_string_buffer(1 << 24)
    r = lib().mscclAmdAlgoJson(xml_path.encode(), rank, nranks, buf, len(buf))
    return r, (json.loads(buf.value.decode()) if r == 0 else None)


def plan_json(xml_files: str, rank: int, nranks: int, coll: int, count: int, dtype: int, op: int,
              in_place: bool) -> dict:
    buf = ctypes.create_string_buffer(1 << 16)
    _check(lib().mscclAmdPlanJson(xml_files.encode(), rank, nranks, coll, count, dtype, op, int(in_place), buf,
                                  len(buf)), "mscclAmdPlanJson")
    return json.loads(buf.value.decode())


def launch_plan_json(xml_files: str, rank: int, nranks: int, one_gpu: bool, coll: int, count: int, dtype: int,
                     op: int, in_place: bool) -> dict:
    """What a communicator launches for one call with init's decisions (plan.cc: planCall): ranks
    all on one GPU (one_gpu) or spread over GPUs; {"kernel", "lowered", "lowerMaxBytes",
    "simpleBuffBytes", ...} (include/msccl_amd.h: mscclAmdLaunchPlanJson)."""
    buf = ctypes.create_string_buffer(1 << 16)
    _check(lib().mscclAmdLaunchPlanJson(xml_files.encode(), rank, nranks, int(one_gpu), coll, count, dtype, op,
                                        int(in_place), buf, len(buf)), "mscclAmdLaunchPlanJson")
    return json.loads(buf.value.decode())


def bootstrap_allgather(uid: bytes, rank: int, nranks: int, payload: bytes) -> bytes:
    u = _uid(uid)
    out = ctypes.create_string_buffer(len(payload) * nranks)
    src = ctypes.create_string_buffer(payload, len(payload))
    _check(lib().mscclAmdBootstrapAllgather(ctypes.byref(u), rank, nranks, src, len(payload), out),
           "mscclAmdBootstrapAllgather")
    return out.raw


class Comm:
    """One rank's communicator (ncclComm_t)."""

    def __init__(self, handle: int):
        self.handle = ctypes.c_void_p(handle)
        L = lib()
        # the collective entry points, looked up once: they sit on the per-call path
        self._ar, self._rs, self._ag = L.ncclAllReduce, L.ncclReduceScatter, L.ncclAllGather

    # ---- creation -------------------------------------------------------------------------
    @staticmethod
    def init_all(devices: Sequence[int]) -> List["Comm"]:
        n = len(devices)
        arr = (ctypes.c_void_p * n)()
        devs = (ctypes.c_int * n)(*devices)
        _check(lib().ncclCommInitAll(arr, n, devs), "ncclCommInitAll")
        return [Comm(arr[i]) for i in range(n)]

    @staticmethod
    def init_rank(nranks: int, uid: bytes, rank: int) -> "Comm":
        h = ctypes.c_void_p()
        _check(lib().ncclCommInitRank(ctypes.byref(h), nranks, _uid(uid), rank), "ncclCommInitRank")
        return Comm(h.value)

    def destroy(self) -> None:
        if self.handle:
            _check(lib().ncclCommDestroy(self.handle), "ncclCommDestroy")
            self.handle = ctypes.c_void_p()

    def abort(self) -> None:
        if self.handle:
            _check(lib().ncclCommAbort(self.handle), "ncclCommAbort")
            self.handle = ctypes.c_void_p()

    # ---- queries ---------------------------------------------------------------------------
    def _q(self, fn, name) -> int:
        v = ctypes.c_int()
        _check(fn(self.handle, ctypes.byref(v)), name)
        return v.value

    @property
    def nranks(self) -> int:
        return self._q(lib().ncclCommCount, "ncclCommCount")

    @property
    def rank(self) -> int:
        return self._q(lib().ncclCommUserRank, "ncclCommUserRank")

    @property
    def device(self) -> int:
        return self._q(lib().ncclCommCuDevice, "ncclCommCuDevice")

    def async_error(self) -> int:
        return self._q(lib().ncclCommGetAsyncError, "ncclCommGetAsyncError")

    def info(self) -> dict:
        buf = ctypes.create_string_buffer(1 << 16)
        _check(lib().mscclAmdCommInfo(self.handle, buf, len(buf)), "mscclAmdCommInfo")
        return json.loads(buf.value.decode())

    def npkit_dump(self, directory: str = None) -> None:
        """Write the NPKit dump now (MSCCL_AMD_NPKIT=1 at init; include/msccl_amd_npkit.h);
        ncclCommDestroy writes it too, into $NPKIT_DUMP_DIR or /tmp/."""
        _check(lib().mscclAmdNpkitDump(self.handle, directory.encode() if directory else None), "mscclAmdNpkitDump")

    def algo_blocks(self, idx: int) -> int:
        return lib().mscclAmdAlgoBlocks(self.handle, idx)

    def trace(self):
        """Device event trace of the most recent launch (MSCCL_AMD_TRACE=1 at init):
        numpy array [slot = tb * maxSplit + sub][event] of TRACE_DTYPE (include/msccl_amd.h)."""
        import numpy as np
        slots, events = ctypes.c_int(), ctypes.c_int()
        _check(lib().mscclAmdTraceRead(self.handle, None, 0, ctypes.byref(slots), ctypes.byref(events)),
               "mscclAmdTraceRead")
        buf = np.zeros(slots.value * events.value, dtype=TRACE_DTYPE)
        _check(lib().mscclAmdTraceRead(self.handle, buf.ctypes.data, buf.nbytes, ctypes.byref(slots),
                                       ctypes.byref(events)), "mscclAmdTraceRead")
        return buf.reshape(slots.value, events.value)

    # ---- user reduction ops (nccl.h.in:153-174) -----------------------------------------------
    def create_premulsum(self, scalar, dtype: int, residence: int = 1) -> int:
        """ncclRedOpCreatePreMulSum.  residence 1 (ncclScalarHostImmediate): `scalar` is bytes of
        the element type (read now); 0 (ncclScalarDevice): `scalar` is a device address read by
        every later kernel."""
        op = ctypes.c_int()
        if residence == 1:
            buf = ctypes.create_string_buffer(bytes(scalar), 8)
            ptr = ctypes.cast(buf, ctypes.c_void_p)
        else:
            ptr = ctypes.c_void_p(scalar)
        _check(lib().ncclRedOpCreatePreMulSum(ctypes.byref(op), ptr, dtype, residence, self.handle),
               "ncclRedOpCreatePreMulSum")
        return op.value

    def destroy_op(self, op: int) -> None:
        _check(lib().ncclRedOpDestroy(op, self.handle), "ncclRedOpDestroy")

    # ---- collectives (pointers are device addresses, stream a hipStream_t or 0) ------------
    def all_reduce(self, send: int, recv: int, count: int, dtype: int, op: int = SUM, stream: int = 0) -> None:
        rc = self._ar(send, recv, count, dtype, op, self.handle, stream)
        if rc:
            raise NcclError(rc, "ncclAllReduce")

    def reduce_scatter(self, send: int, recv: int, recvcount: int, dtype: int, op: int = SUM, stream: int = 0) -> None:
        rc = self._rs(send, recv, recvcount, dtype, op, self.handle, stream)
        if rc:
            raise NcclError(rc, "ncclReduceScatter")

    def all_gather(self, send: int, recv: int, sendcount: int, dtype: int, stream: int = 0) -> None:
        rc = self._ag(send, recv, sendcount, dtype, self.handle, stream)
        if rc:
            raise NcclError(rc, "ncclAllGather")

    def all_to_all(self, send: int, recv: int, count: int, dtype: int, stream: int = 0) -> None:
        _check(lib().ncclAllToAll(send, recv, count, dtype, self.handle, stream), "ncclAllToAll")

    def custom(self, send: int, recv: int, count: int, dtype: int, algo_index: int, stream: int = 0) -> None:
        _check(lib().ncclCustomCollective(send, recv, count, dtype, algo_index, self.handle, stream),
               "ncclCustomCollective")


class group:
    """ncclGroupStart / ncclGroupEnd (nccl.h.in:369-380) as a context manager (a class, not a
    generator: it sits on the per-call path of small collectives)."""
    __slots__ = ()

    def __enter__(self):
        rc = lib().ncclGroupStart()
        if rc:
            raise NcclError(rc, "ncclGroupStart")
        return self

    def __exit__(self, *exc):
        rc = lib().ncclGroupEnd()
        if rc:
            raise NcclError(rc, "ncclGroupEnd")
        return False


def torch_dtype_code(t) -> int:
    import torch
    m = {torch.int8: INT8, torch.uint8: UINT8, torch.int32: INT32, torch.int64: INT64, torch.float16: FLOAT16,
         torch.float32: FLOAT32, torch.float64: FLOAT64, torch.bfloat16: BFLOAT16}
    if hasattr(torch, "uint32"):
        m[torch.uint32] = UINT32
    if hasattr(torch, "uint64"):
        m[torch.uint64] = UINT64
    return m[t]

"""ORACLE (test infrastructure only) — MSCCL algorithm selection and per-call chunk math.

Restates, on the host, what decides the interpreter's work split (and therefore the
association order of every reduction):
  ArgsCheck                    /root/reference/src/misc/argcheck.cc:36-80
  in-place / totalCount        graph/tuning.cc:312-342   (mscclInPlaceTotalCountHelper)
  algorithm match              graph/tuning.cc:344-382   (ncclTopoGetMSCCLAlgo)
  threads                      graph/tuning.cc:14-32,78-85; enqueue.cc:486-523 (+32 for Simple)
  chunk math / maxAllowedCount enqueue.cc:591-734        (computeColl MSCCL parts)
  scratch check                enqueue.cc:580-589
  interpreter chunking         collectives/device/msccl_interpreter.h:79-113
Buffer sizes: init.cc:451-472 (LL 524288, LL128 4915200, Simple 4 MiB) and
NCCL_LL_BUFFSIZE / NCCL_LL128_BUFFSIZE / NCCL_BUFFSIZE.
"""
from __future__ import annotations

import dataclasses
import os
from typing import List, Optional

from . import loader as L
from . import numerics as N

NCCL_STEPS = 8
LL_MAX_NTHREADS = 512
SIMPLE_MAX_NTHREADS = 512
LL128_MAX_NTHREADS = 640
REF_WARP = 32
MSCCL_CHUNKSTEPS = NCCL_STEPS // 2
DEFAULT_BUFFSIZES = [8 * 512 * NCCL_STEPS * 16, 120 * 640 * NCCL_STEPS * 8, 1 << 22]


def buff_sizes() -> List[int]:
    out = list(DEFAULT_BUFFSIZES)
    for i, k in enumerate(("NCCL_LL_BUFFSIZE", "NCCL_LL128_BUFFSIZE", "NCCL_BUFFSIZE")):
        v = os.environ.get(k)
        if v is not None:
            out[i] = int(v, 0)
    return out


def _env_nthreads(name: str, lo: int, hi: int, default: int) -> int:
    # tuning.cc:14-32
    v = os.environ.get(name)
    nt = int(v, 0) if v is not None else -2
    if nt > 0:
        if nt % REF_WARP != 0:
            return hi
        if nt > hi:
            return hi
        if nt < lo:
            return lo
        return nt
    return default


def max_threads(proto: int) -> int:
    if proto == L.PROTO_SIMPLE:
        return _env_nthreads("NCCL_NTHREADS", 2 * REF_WARP, SIMPLE_MAX_NTHREADS, SIMPLE_MAX_NTHREADS)
    if proto == L.PROTO_LL:
        return _env_nthreads("NCCL_NTHREADS", 2 * REF_WARP, LL_MAX_NTHREADS, LL_MAX_NTHREADS)
    return _env_nthreads("NCCL_LL128_NTHREADS", LL128_MAX_NTHREADS // 4, LL128_MAX_NTHREADS, LL128_MAX_NTHREADS)


@dataclasses.dataclass
class Call:
    coll: int            # ncclFunc_t
    count: int           # user count (recvcount for RS, sendcount for AG)
    dtype: int           # ncclDataType_t
    op: int              # ncclRedOp_t
    nranks: int
    rank: int
    in_place: bool


@dataclasses.dataclass
class Plan:
    algo_index: int
    proto: int
    nthreads: int          # reference thread count (decides LL minChunk / Simple rounding / small path)
    count: int             # interpreter args->count (bytes for AllGather)
    dtype: int             # interpreter element type (int8 for AllGather)
    size_multiplier: int
    nbytes: int
    max_allowed_count: int
    ncpl: int
    op: int = 0


def args_check(c: Call):
    """argcheck.cc:44-51: returns (interpreter count, interpreter dtype, nBytes)."""
    nbytes = c.count * N.type_size(c.dtype)
    count, dtype = c.count, c.dtype
    if c.coll in (L.ALLGATHER, L.BROADCAST, L.ALLTOALL):
        count, dtype = nbytes, 0
    if c.coll in (L.ALLGATHER, L.REDUCE_SCATTER, L.ALLTOALL):
        nbytes *= c.nranks
    return count, dtype, nbytes


def total_count(c: Call, count: int) -> int:
    # tuning.cc:312-342 (count is the post-ArgsCheck count)
    if c.coll in (L.ALLTOALL, L.ALLGATHER, L.REDUCE_SCATTER):
        return count * c.nranks
    return count


def select(algos: List[L.Algorithm], c: Call, registrations=None) -> Optional[int]:
    """tuning.cc:344-382. Returns the algorithm index or None (reference falls back to ring/tree)."""
    if c.op not in (N.SUM, N.PROD, N.MAX, N.MIN):
        return None
    count, _, nbytes = args_check(c)
    tc = total_count(c, count)
    if registrations:
        for reg in registrations:
            if reg["minBytes"] <= nbytes and (nbytes < reg["maxBytes"] or reg["maxBytes"] == -1):
                a = algos[reg["algoIndex"]]
                if (a.valid and a.coll == c.coll and int(c.in_place) == a.inplace and a.ngpus == c.nranks
                        and tc % a.nchunksperloop == 0):
                    return reg["algoIndex"]
        return None
    for i, a in enumerate(algos):
        if (a.valid and a.coll == c.coll and int(c.in_place) == a.inplace and a.ngpus == c.nranks
                and tc % a.nchunksperloop == 0 and a.minBytes <= nbytes < a.maxBytes):
            return i
    return None


def make_plan(algos: List[L.Algorithm], c: Call, algo_index: int, proto: Optional[int] = None) -> Plan:
    a = algos[algo_index]
    proto = a.proto if proto is None else proto
    count, dtype, nbytes = args_check(c)
    nt = max_threads(proto)
    if a.nthreads > 0:
        nt = min(nt, a.nthreads)
    if proto == L.PROTO_SIMPLE:
        nt += REF_WARP
    bs = buff_sizes()
    step_size = bs[proto] // NCCL_STEPS
    chunk_steps = MSCCL_CHUNKSTEPS if proto == L.PROTO_SIMPLE else 1
    chunk_size = step_size * chunk_steps
    chunk_eff = chunk_size
    if proto == L.PROTO_LL:
        chunk_eff //= 2
    if proto == L.PROTO_LL128:
        chunk_eff = (chunk_size // 16) * 15
    if nbytes % a.nchunksperloop != 0:
        raise ValueError("MSCCL algorithm needs the input buffer to be divisible by %d" % a.nchunksperloop)
    if proto == L.PROTO_SIMPLE and chunk_size % ((nt - REF_WARP) * 8 // N.type_size(dtype)) != 0:
        raise ValueError("chunkSize should be divisible by (nthreads-WARP_SIZE)")
    mac = 0
    if nbytes > 0:
        mac = max(1, chunk_eff // -(-nbytes // a.nchunksperloop))
    if mac == 0:
        raise ValueError("Max allowed count is 0")
    mac = min(mac, 71)
    mult = c.nranks if c.coll in (L.REDUCE_SCATTER, L.ALLGATHER, L.ALLTOALL) else 1
    return Plan(algo_index, proto, nt, count, dtype, mult, nbytes, mac, a.nchunksperloop, c.op)


def chunking(plan: Plan, ts: int):
    """msccl_interpreter.h:79-113: yields (iter, gridOffset, nelem) for each outer iteration."""
    bs = buff_sizes()
    if plan.proto == L.PROTO_LL:
        byte_per_step = bs[0] // NCCL_STEPS // 2
        min_chunk = plan.nthreads * (8 // ts)
    elif plan.proto == L.PROTO_LL128:
        byte_per_step = (bs[1] // NCCL_STEPS) * 15 // 16
        grain = 8 * 15 * 8 // 16
        min_chunk = plan.nthreads * (grain // ts) // 2
    else:
        byte_per_step = bs[2] // NCCL_STEPS
        min_chunk = 0
    chunk_size = int(byte_per_step // ts * (MSCCL_CHUNKSTEPS if plan.proto == L.PROTO_SIMPLE else 1))
    size_per = (plan.count * plan.size_multiplier) // plan.ncpl
    grid, it = 0, 0
    while grid < size_per:
        if plan.proto == L.PROTO_SIMPLE:
            real = min(chunk_size, size_per - grid)
            unit = (plan.nthreads - REF_WARP) * 8 // ts
            real = -(-real // unit) * unit
        else:
            real = min(chunk_size, -(-(size_per - grid) // min_chunk) * min_chunk)
        real = int(real)
        nelem = min(real, size_per - grid)
        yield it, grid, nelem, size_per
        grid += chunk_size
        it += 1

"""ORACLE (test infrastructure only) — CPU restatement of the reference's NCCL ring collectives,
the path a call takes when no MSCCL algorithm matches (enqueue.cc:461-476 falls back to ring).

Restated from the reference device code:
  AllReduce      /root/reference/src/collectives/device/all_reduce.h:14-100     (runRing)
  ReduceScatter  /root/reference/src/collectives/device/reduce_scatter.h:13-67  (runRing)
  AllGather      /root/reference/src/collectives/device/all_gather.h:13-78      (runRing)
and the host chunk math:
  chunkSize      Proto::calcBytePerStep (primitives.h:31-51) x CHUNKSTEPS (4 for Simple)
  lastChunkSize  enqueue.cc:653-658 (LL ring: remainder / (nChannels * nRanks), aligned to nThreads*8 B)
  nThreads       enqueue.cc:486-523 (LL 512; Simple 512 + one sync warp, 516-517)
Primitive values: LL recv-reduce fn(peer, local) (prims_ll.h:282-287); Simple fn(local, peer)
(common_kernel.h:490-555, srcs = [local, peer]).  A primitive with nelem <= 0 moves nothing.
PreMulSum / SumPostDiv (ncclAvg, user ops): every value loaded from the user's input is scaled
first (prims_ll.h:280, prims_simple.h:209-211 PreOpN), and the final reduction of AllReduce (rrcs,
all_reduce.h:84) and ReduceScatter (rrc, reduce_scatter.h:65) applies the postOp.

Where the reference consults its topology search and tuning model (graph/search.cc,
tuning.cc:77-309, enqueue.cc:486-515), this build decides as follows; ring_params() states it and
msccl_amd/csrc/plan.cc (makeRingPlan) mirrors it:
  * the ring order is the rank order: ringRanks of rank r = [r, r+1, ..., r-1] (mod n);
  * channels = min(32, max(1, nBytes >> 18)) (MSCCL_AMD_RING_CHANNELS forces it);
  * LL when nBytes <= 512 KiB, else Simple (NCCL_PROTO masks them; LL128 is not used here);
  * nThreads is not reduced for small messages (the reference halves it below its thresholds);
  * AllReduce calls of at most MSCCL_AMD_TREE_MAX_BYTES (default 16 KiB per rank; 512 KiB, the LL
    range, where the flat tree runs them: LL, ops Sum..Min, 2..16 ranks), or all of them when
    NCCL_ALGO enables Tree but not Ring, take the tree: the reference's runTreeSplit
    (all_reduce.h:174-276) on a chain in rank order (root 0, parent r-1, child r+1), with
    computeColl's tree chunk math (enqueue.cc:634-644; tree depth = nranks) and the kernel's
    loopSize > size shrink (all_reduce.h:121-122).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import loader as L
from . import numerics as N
from . import plan as P

RING_MAX_CHANNELS = 32
RING_LL_MAX_BYTES = 512 << 10
REF_WARP = 32


def _proto_enabled(name: str) -> bool:
    s = os.environ.get("NCCL_PROTO")
    if s is None:
        return True
    inv = s.startswith("^")
    names = [x.strip().lower() for x in (s[1:] if inv else s).split(",")]
    found = name.lower() in names
    return not found if inv else found


def _algo_enabled(name: str) -> bool:
    s = os.environ.get("NCCL_ALGO")
    if s is None:
        return True
    inv = s.startswith("^")
    names = [x.strip().lower() for x in (s[1:] if inv else s).split(",")]
    found = name.lower() in names
    return not found if inv else found


def tree_params(rp: dict, nranks: int) -> dict:
    """The tree variant of a fallback AllReduce (plan.cc: makeTreePlan)."""
    ts, C, size, nbytes = rp["ts"], rp["channels"], rp["size"], rp["nbytes"]
    bs = P.buff_sizes()
    if rp["proto"] == L.PROTO_LL:
        nthreads = P.max_threads(L.PROTO_LL)
        chunk = bs[0] // P.NCCL_STEPS * 8 // 16 // ts
        min_chunk = nthreads * 8 // ts
    else:
        nthreads = P.max_threads(L.PROTO_SIMPLE) + REF_WARP + 3 * REF_WARP
        cb = bs[2] // P.NCCL_STEPS
        depth = nranks
        while nbytes // (C * cb) < depth * 8 and cb > 131072:
            cb //= 2
        while nbytes // (C * cb) < depth * 4 and cb > 65536:
            cb //= 2
        while nbytes // (C * cb) < depth and cb > 32768:
            cb //= 2
        chunk = cb // ts
        min_chunk = (nthreads - 2 * REF_WARP) * 8 * (8 // ts)
    if C * chunk > size:
        chunk = -(-size // (C * min_chunk)) * min_chunk
    out = dict(rp)
    out.update({"algo": "tree", "nthreads": nthreads, "chunk": chunk, "min_chunk": min_chunk})
    return out


def ring_params(coll: int, count: int, dtype: int, nranks: int, op: int = 0) -> Optional[dict]:
    """Host-side decisions for one fallback call: interpreter dtype/size (elements of one rank's
    block), nBytes, proto, channels, nthreads, chunkSize and, for LL ReduceScatter/AllGather,
    lastChunkSize (elements)."""
    nbytes = count * N.type_size(dtype)
    size, dt = count, dtype
    if coll == L.ALLGATHER:                      # ArgsCheck: AllGather moves bytes (argcheck.cc:44-51)
        size, dt = nbytes, 0
    if coll in (L.ALLGATHER, L.REDUCE_SCATTER):
        nbytes *= nranks
    ts = N.type_size(dt)
    ll_ok, simple_ok = _proto_enabled("LL"), _proto_enabled("Simple")
    if not ll_ok and not simple_ok:
        return None
    proto = L.PROTO_LL if (ll_ok and (nbytes <= RING_LL_MAX_BYTES or not simple_ok)) else L.PROTO_SIMPLE
    forced = int(os.environ.get("MSCCL_AMD_RING_CHANNELS", "0") or 0)
    chans = forced if forced > 0 else max(1, nbytes >> 18)
    chans = max(1, min(RING_MAX_CHANNELS, chans))
    bs = P.buff_sizes()
    if proto == L.PROTO_LL:
        nthreads = P.max_threads(L.PROTO_LL)
        chunk = bs[0] // P.NCCL_STEPS // 2 // ts
        min_chunk = nthreads * 8 // ts
    else:
        nthreads = P.max_threads(L.PROTO_SIMPLE) + REF_WARP
        chunk = bs[2] // P.NCCL_STEPS // ts * P.MSCCL_CHUNKSTEPS
        min_chunk = (nthreads - REF_WARP) * 8 // ts
    last = 0
    if proto == L.PROTO_LL and coll in (L.REDUCE_SCATTER, L.ALLGATHER):
        step = bs[0] // P.NCCL_STEPS
        slice_size = step * 8 // 16
        loop = chans * nranks * slice_size
        last = -(-(nbytes - (nbytes // loop) * loop) // (chans * nranks))
        align = nthreads * 8
        last = -(-last // align) * align
        last //= ts
    rp = {"coll": coll, "size": size, "dtype": dt, "nbytes": nbytes, "proto": proto, "channels": chans,
          "nthreads": nthreads, "chunk": chunk, "min_chunk": min_chunk, "last_chunk": last, "ts": ts,
          "algo": "ring"}
    tree_max = int(os.environ.get("MSCCL_AMD_TREE_MAX_BYTES", "-1") or -1)
    if tree_max < 0:
        flat = int(os.environ.get("MSCCL_AMD_TREE_FLAT", "1") or 1) != 0 and proto == L.PROTO_LL and \
            op <= 3 and 2 <= nranks <= 16
        tree_max = RING_LL_MAX_BYTES if flat else 16384 * nranks
    ring_ok, tree_ok = _algo_enabled("Ring"), _algo_enabled("Tree")
    if coll == L.ALLREDUCE and tree_ok and (not ring_ok or count * N.type_size(dtype) <= tree_max):
        return tree_params(rp, nranks)
    if not ring_ok:
        return None
    return rp


def tree_ops(rp: dict, rank: int, n: int, bid: int):
    """Channel bid // 2 of the chain tree: bid even reduces up, bid odd broadcasts down.  Yields
    (kind, src_off, dst_off, nelem, recv_peer, send_peer)."""
    size, C, chunk = rp["size"], rp["channels"], rp["chunk"]
    c, up = bid // 2, bid % 2 == 0
    parent, child = rank - 1, rank + 1 if rank + 1 < n else -1
    grid = 0
    while grid < size:
        off = grid + c * chunk
        ne = max(0, min(chunk, size - off))
        if up:
            if rank == 0:
                yield ("rrcs", off, off, ne, child, child)          # recvReduceCopySend, postOp
            elif child < 0:
                yield ("s", off, None, ne, -1, parent)
            else:
                yield ("rrs", off, None, ne, child, parent)
        elif rank > 0:
            if child < 0:
                yield ("r", None, off, ne, parent, -1)
            else:
                yield ("rcs", None, off, ne, parent, child)         # directRecvCopySend
        grid += C * chunk


def ops(rp: dict, rank: int, n: int, bid: int):
    """The reference's op sequence of channel `bid` on `rank`: yields (kind, src_off, dst_off, nelem);
    kind is one of s, rrs, rrcs, rcs, r, rrc, cs (copy + send, AllGather out of place)."""
    coll, size, proto, C, chunk = rp["coll"], rp["size"], rp["proto"], rp["channels"], rp["chunk"]
    ring = [(rank + k) % n for k in range(n)]
    if coll == L.ALLREDUCE:
        loop = C * n * chunk
        grid = 0
        while grid < size:
            if proto == L.PROTO_SIMPLE:                                   # all_reduce.h:43-46
                real = min(chunk, -(-(size - grid) // (C * n)))
                unit = rp["min_chunk"]
                real = -(-real // unit) * unit
            else:                                                         # all_reduce.h:48
                mc = rp["min_chunk"]
                real = min(chunk, -(-(size - grid) // (C * n * mc)) * mc)

            def off(c):                                                   # all_reduce.h:51-56
                if proto == L.PROTO_SIMPLE:
                    return grid + bid * n * real + c * real
                return grid + (c * C + bid) * real

            def ne(o):
                return max(0, min(real, size - o))
            c = ring[n - 1]                                               # step 0 (66-69)
            yield ("s", off(c), None, ne(off(c)))
            for j in range(2, n):                                         # 72-77
                c = ring[n - j]
                yield ("rrs", off(c), None, ne(off(c)))
            c = ring[0]                                                   # 81-84
            yield ("rrcs", off(c), off(c), ne(off(c)))
            for j in range(1, n - 1):                                     # 87-92
                c = ring[n - j]
                yield ("rcs", None, off(c), ne(off(c)))
            c = ring[1]                                                   # 95-98
            yield ("r", None, off(c), ne(off(c)))
            grid += loop
    else:
        loop = C * chunk
        grid = 0
        while grid < size:
            if proto == L.PROTO_SIMPLE:                                   # reduce_scatter.h:33-36
                real = min(chunk, -(-(size - grid) // C))
                unit = rp["min_chunk"]
                real = -(-real // unit) * unit
            else:                                                         # reduce_scatter.h:37-38
                real = rp["last_chunk"] if size - grid < loop else chunk
            co = grid + bid * real
            nelem = max(0, min(real, size - co))
            if coll == L.REDUCE_SCATTER:                                  # reduce_scatter.h:50-65
                yield ("s", co + ring[n - 1] * size, None, nelem)
                for j in range(2, n):
                    yield ("rrs", co + ring[n - j] * size, None, nelem)
                yield ("rrc", co + ring[0] * size, co, nelem)
            else:                                                         # all_gather.h:52-75
                yield ("cs", co, co + ring[0] * size, nelem)
                for j in range(1, n - 1):
                    yield ("rcs", None, co + ring[n - j] * size, nelem)
                yield ("r", None, co + ring[1] * size, nelem)
            grid += loop


def run(coll: int, count: int, dtype: int, op: int, inputs: Sequence[np.ndarray],
        outputs: Sequence[Optional[np.ndarray]], in_place: bool, arg: int = 0):
    """Run the ring fallback on all ranks.  inputs/outputs as oracle/sim.run (element type of the
    call; AllGather buffers may be any type, they are moved as bytes).  For in-place calls pass
    outputs[r]=None except for AllGather, whose output buffer holds the input at rank*count.
    Returns (outputs, params)."""
    n = len(inputs)
    rp = ring_params(coll, count, dtype, n, op)
    size, dt = rp["size"], rp["dtype"]
    ins, outs = [], []
    for r in range(n):
        inp = inputs[r]
        if coll == L.ALLGATHER:
            inp = inp.view(np.int8)
        if in_place:
            if coll == L.REDUCE_SCATTER:
                out = inp[r * size:(r + 1) * size]
            elif coll == L.ALLGATHER:
                out = outputs[r].view(np.int8)
                out[r * size:(r + 1) * size] = inp[:size]
                inp = out[r * size:(r + 1) * size]
            else:
                out = inp
        else:
            out = outputs[r].view(np.int8) if coll == L.ALLGATHER else outputs[r]
        ins.append(inp)
        outs.append(out)
    fifos: Dict[Tuple[int, int, int], List[np.ndarray]] = {}

    def steps(r, bid):
        if rp["algo"] == "tree":
            for kind, so, do, ne, src, dst in tree_ops(rp, r, n, bid):
                yield kind, so, do, ne, (bid // 2, src, r), (bid // 2, r, dst)
        else:
            for kind, so, do, ne in ops(rp, r, n, bid):
                yield kind, so, do, ne, (bid, (r - 1) % n, r), (bid, r, (r + 1) % n)

    def prog(r, bid):
        for kind, so, do, ne, rkey, skey in steps(r, bid):
            msg = None
            if kind in ("rrs", "rrcs", "rcs", "r", "rrc"):
                key = rkey
                while not fifos.get(key):
                    yield False
                msg = fifos[key].pop(0)
                assert len(msg) == ne, (kind, len(msg), ne)
            if kind == "cs":
                # all_gather.h:56-60: in place the data already sits in the output (directSend)
                v = outs[r][do:do + ne].copy() if in_place else ins[r][so:so + ne].copy()
                if not in_place:
                    outs[r][do:do + ne] = v
                fifos.setdefault(skey, []).append(v)
            elif kind == "s":
                v = ins[r][so:so + ne].copy()
                if coll != L.ALLGATHER:
                    v = N.pre_op(op, dt, v, arg)
                fifos.setdefault(skey, []).append(v)
            elif kind in ("rrs", "rrcs", "rrc"):
                local = N.pre_op(op, dt, ins[r][so:so + ne].copy(), arg)
                if rp["proto"] == L.PROTO_SIMPLE:
                    v = N.apply(op, dt, local, msg)
                else:
                    v = N.apply(op, dt, msg, local)
                if kind in ("rrcs", "rrc"):
                    v = N.post_op(op, dt, v, arg)
                if kind in ("rrcs", "rrc"):
                    outs[r][do:do + ne] = v
                if kind in ("rrs", "rrcs"):
                    fifos.setdefault(skey, []).append(v)
            elif kind == "rcs":
                outs[r][do:do + ne] = msg
                fifos.setdefault(skey, []).append(msg)
            else:  # r
                outs[r][do:do + ne] = msg
            yield True

    nb = rp["channels"] * (2 if rp["algo"] == "tree" else 1)
    live = [prog(r, b) for r in range(n) for b in range(nb)]
    while live:
        progress, nxt_live = False, []
        for g in live:
            done = False
            while True:
                try:
                    p = next(g)
                except StopIteration:
                    done, progress = True, True
                    break
                if not p:
                    break
                progress = True
            if not done:
                nxt_live.append(g)
        live = nxt_live
        if live and not progress:
            raise RuntimeError("ring oracle deadlock")
    if coll == L.ALLGATHER:
        outs = [o.view(N.storage(dtype)) for o in outs]
    return outs, rp

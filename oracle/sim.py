"""ORACLE (test infrastructure only) — CPU simulator of the MSCCL schedule interpreter.

Executes every rank's thread-block program on host numpy buffers with the exact data
semantics of the reference's device path:
  interpreter loop      /root/reference/src/collectives/device/msccl_interpreter.h:66-205
                        (gridOffset iterations x transfers; count split by mscclMaxAllowedCount;
                         offsets (xmlOff + c) * sizePerMscclChunk + gridOffset; dependency flags
                         COMPUTE_FLAG(workIndex, iter, step); `ra` and unknown types end the tb)
  LL primitives         device/prims_ll.h:247-380
                        recv-reduce: fn(peer, local)              (prims_ll.h:282-287)
                        reduce:      acc = d; acc = fn(acc, s_i)  (prims_ll.h:347-362)
  LL128 primitives      device/prims_ll128.h:184-425
                        recv-reduce: fn(peer, local)              (prims_ll128.h:235-236)
                        reduce:      acc = d; acc = fn(s_i, acc)  (prims_ll128.h:381-392)
  Simple primitives     device/prims_simple.h:131-281, common_kernel.h:490-690
                        recv-reduce: fn(local, peer)              (srcs = [local, peer], left fold)
                        reduce:      ((s0 (+) s1) ...) (+) d      (dst appended last, prims_simple.h:258-263)
  small reduce path     msccl_interpreter.h:157-170: thisNelem < nthreads -> per element
                        o = d; o = fn(s_r, o) for every protocol
  send/recv matching    per (channel, sender, receiver) FIFO, one primitive call = one FIFO message
                        (one LL step / one Simple chunk), consumed in order.
Thread blocks are run as cooperative coroutines; a transfer blocks on its dependency flags and
on an empty receive FIFO.  Sends never block (the FIFO depth only affects timing, not values).
A schedule that cannot make progress raises SimDeadlock (this is also how a malformed XML shows).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import loader as L
from . import numerics as N
from . import plan as P


class SimDeadlock(RuntimeError):
    pass


class SimError(RuntimeError):
    pass


def _tb_program(algo: L.Algorithm, bid: int, rank: int, plan: P.Plan, bufs, fifos, flags, stats):
    """Generator: yields False when blocked, True after progress; returns when the tb is done."""
    tb = algo.tbs[bid]
    ts = N.type_size(plan.dtype)
    dt = plan.dtype
    op = plan.op
    proto = plan.proto
    nthreads = plan.nthreads
    mac = plan.max_allowed_count
    for it, grid, nelem, size_per in P.chunking(plan, ts):
        step = 0
        for tr in tb.transfers:
            if tr.numDeps > 0:
                for d in range(tr.numDeps):
                    dbid = tb.depBid[tr.depPtr + d]
                    dstep = tb.depStep[tr.depPtr + d]
                    goal = (it, dstep)
                    while flags[rank].get(dbid, (-1, -1)) < goal:
                        yield False
                step += tr.numDeps - 1
            src = bufs[rank][tr.srcbuf]
            dst = bufs[rank][tr.dstbuf]
            c = 0
            while c < tr.count:
                srcoff = grid + (tr.srcoff + c) * size_per
                dstoff = grid + (tr.dstoff + c) * size_per
                this_count = min(mac, tr.count - c)
                n = nelem * this_count
                t = tr.type
                if t in (L.RECV, L.RCS, L.RRS, L.RRC, L.RRCS):
                    key = (tb.chan, tb.recv, rank)
                    while not fifos.get(key):
                        yield False
                    msg = fifos[key].pop(0)
                    if len(msg) != max(n, 0):
                        raise SimError("rank %d tb %d: recv of %d elements got a message of %d"
                                       % (rank, bid, n, len(msg)))
                    stats["recv_bytes"] += len(msg) * ts
                if t == L.SEND:
                    _send(fifos, (tb.chan, rank, tb.send), src[srcoff:srcoff + n], stats, ts)
                elif t == L.RECV:
                    dst[dstoff:dstoff + n] = msg
                elif t == L.RCS:
                    dst[dstoff:dstoff + n] = msg
                    _send(fifos, (tb.chan, rank, tb.send), msg, stats, ts)
                elif t in (L.RRS, L.RRC, L.RRCS):
                    local = src[srcoff:srcoff + n].copy()
                    if proto == L.PROTO_SIMPLE:
                        v = N.apply(op, dt, local, msg)
                    else:
                        v = N.apply(op, dt, msg, local)
                    if t in (L.RRC, L.RRCS):
                        dst[dstoff:dstoff + n] = v
                    if t in (L.RRS, L.RRCS):
                        _send(fifos, (tb.chan, rank, tb.send), v, stats, ts)
                elif t == L.CPY:
                    dst[dstoff:dstoff + n] = src[srcoff:srcoff + n].copy()
                elif t == L.RE:
                    nred = tr.numReds
                    srcs = []
                    for r in range(nred):
                        so = grid + (tb.redSrcOff[tr.redPtr + r] + c) * size_per
                        srcs.append(src[so:so + n].copy())
                    d = dst[dstoff:dstoff + n].copy()
                    if n < nthreads or proto != L.PROTO_SIMPLE:
                        # LL / LL128 order, and the small path of every protocol: dst first;
                        # LL folds fn(acc, s) (prims_ll.h:352-358), LL128 and the small path
                        # fn(s, acc) (prims_ll128.h:381-392, msccl_interpreter.h:163-166)
                        acc = d
                        for s in srcs:
                            if n < nthreads or proto == L.PROTO_LL128:
                                acc = N.apply(op, dt, s, acc)
                            else:
                                acc = N.apply(op, dt, acc, s)
                    else:
                        acc = srcs[0]
                        for s in srcs[1:]:
                            acc = N.apply(op, dt, acc, s)
                        acc = N.apply(op, dt, acc, d)
                    dst[dstoff:dstoff + n] = acc
                    if c == 0:
                        step += nred - 1
                else:
                    return  # MSCCL_RES_ADD and unknown types end the thread block (interpreter.h:195-196)
                c += mac
            if tr.hasDep:
                flags[rank][bid] = (it, step)
            step += 1
            yield True


def _send(fifos, key, data, stats, ts):
    fifos.setdefault(key, []).append(np.array(data, copy=True))
    stats["send_bytes"] += len(data) * ts


def run(algos_by_rank: Sequence[L.Algorithm], plan: P.Plan, inputs: Sequence[np.ndarray],
        outputs: Sequence[Optional[np.ndarray]], coll: int, in_place: bool, scratch_elems: Optional[int] = None):
    """Run one collective on all ranks.

    algos_by_rank[r] is the algorithm as loaded for rank r.  inputs[r]/outputs[r] are flat
    numpy arrays in the interpreter's element type (bytes for AllGather).  For in-place
    calls pass outputs[r]=None: the output aliases the input as the reference defines it
    (AllReduce: same buffer; ReduceScatter: out = in[rank*count:]; AllGather: in = out[rank*count:]).
    Returns (outputs, stats).
    """
    n = len(algos_by_rank)
    bufs: List[Dict[int, np.ndarray]] = []
    ts = N.type_size(plan.dtype)
    size_per = (plan.count * plan.size_multiplier) // plan.ncpl
    outs = []
    for r in range(n):
        a = algos_by_rank[r]
        inp = inputs[r]
        if in_place:
            if coll == L.REDUCE_SCATTER:
                out = inp[r * plan.count:(r + 1) * plan.count]
            elif coll == L.ALLGATHER:
                out = outputs[r]
                out[r * plan.count:(r + 1) * plan.count] = inp[:plan.count]
                inp = out[r * plan.count:(r + 1) * plan.count]
            else:
                out = inp
        else:
            out = outputs[r]
        nscr = scratch_elems if scratch_elems is not None else max(a.nScratchChunks * size_per, 1)
        scratch = np.zeros(nscr, dtype=inp.dtype)
        bufs.append({L.INPUT: inp, L.OUTPUT: out, L.SCRATCH: scratch})
        outs.append(out)
    plan_op = plan
    fifos: Dict[Tuple[int, int, int], List[np.ndarray]] = {}
    flags: List[Dict[int, Tuple[int, int]]] = [dict() for _ in range(n)]
    stats = {"send_bytes": 0, "recv_bytes": 0}
    progs = []
    for r in range(n):
        for b in range(algos_by_rank[r].nBlocks):
            progs.append(_tb_program(algos_by_rank[r], b, r, plan_op, bufs, fifos, flags, stats))
    live = list(progs)
    while live:
        progress = False
        nxt = []
        for g in live:
            done = False
            while True:
                try:
                    p = next(g)
                except StopIteration:
                    done = True
                    progress = True
                    break
                if not p:
                    break
                progress = True
            if not done:
                nxt.append(g)
        live = nxt
        if live and not progress:
            raise SimDeadlock("schedule cannot make progress (%d thread blocks blocked)" % len(live))
    leftover = {k: len(v) for k, v in fifos.items() if v}
    if leftover:
        raise SimError("unconsumed FIFO messages: %r" % leftover)
    return outs, stats


def allreduce_reference(inputs: Sequence[np.ndarray], dt: int, op: int) -> np.ndarray:
    """Naive left fold x_0 (+) x_1 (+) ... used only to bound the schedule result (1 ulp gate)."""
    acc = inputs[0].copy()
    for x in inputs[1:]:
        acc = N.apply(op, dt, acc, x)
    return acc

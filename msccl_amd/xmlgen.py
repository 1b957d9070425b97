"""MSCCL XML schedule generators (the msccl-tools algorithms the benchmarks need).

msccl-tools (the Python DSL that emits MSCCL XML) is not installed in this image, so the
schedules used by the benchmarks and tests are generated here.  The output is the
msccl-tools XML dialect the reference loader accepts (graph/topo.cc:759-1193): one <algo>
with <gpu>/<tb>/<step> children, steps numbered densely from 0, `nop` steps carrying extra
dependencies and chained `re` steps that the loader fuses into one multi-source reduction.

allreduce_allpairs reproduces the structure of msccl-tools' "allreduce_pairs" as shipped by
RCCL (/opt/rocm/share/rccl/msccl-algorithms/allreduce-allpairs-8n-ll-32tb.xml): for n ranks and
I instances (channels) the loop has I*n*n chunks, rank r owns chunks [k*n*n + r*n, +n) of
instance k; thread block (k, peer p) sends the peer's n chunks to the peer's scratch, receives the
peer's copy of its own chunks, reduces owned chunk p from all scratch slots and then exchanges
the reduced chunks; thread block k (one per instance) reduces owned chunk r.  For n=8, I=4 the
generated file is step-for-step the shipped 32-tb schedule (checked in tests).
"""
from __future__ import annotations

import io
from typing import Dict, List, Optional, Tuple

Step = Tuple[str, str, int, str, int, int, int, int, int]  # type, srcbuf, srcoff, dstbuf, dstoff, cnt, depid, deps, hasdep


class _Tb:
    def __init__(self, tid: int, send: int, recv: int, chan: int):
        self.id, self.send, self.recv, self.chan = tid, send, recv, chan
        self.steps: List[Step] = []

    def add(self, typ, srcbuf="i", srcoff=-1, dstbuf="o", dstoff=-1, cnt=0, depid=-1, deps=-1, hasdep=0) -> int:
        self.steps.append((typ, srcbuf, srcoff, dstbuf, dstoff, cnt, depid, deps, hasdep))
        return len(self.steps) - 1

    def nop(self, depid: int, deps: int) -> int:
        return self.add("nop", "i", -1, "o", -1, 0, depid, deps, 0)



# Default maxBytes of the schedules that use scratch (two-phase all-pairs, one-shot): the runtime
# allocates scratch for maxBytes at init (init.cc:809-835), so an unbounded default would pin the
# 8 GiB MSCCL_AMD_MAX_SCRATCH cap per rank.  Larger calls take the fallback unless the caller
# passes max_bytes.  Scratch-free schedules (pair one-shot, ring) stay unbounded.
SCRATCH_SCHEDULE_MAX_BYTES = 1 << 30

def _emit(name: str, proto: str, nchannels: int, ncpl: int, ngpus: int, coll: str, inplace: bool,
          gpus: Dict[int, Tuple[int, int, int, List[_Tb]]], min_bytes: Optional[int], max_bytes: Optional[int],
          nthreads: Optional[int] = None) -> str:
    o = io.StringIO()
    attrs = ('name="%s" proto="%s" nchannels="%d" nchunksperloop="%d" ngpus="%d" coll="%s" inplace="%d" '
             'outofplace="%d"' % (name, proto, nchannels, ncpl, ngpus, coll, int(inplace), int(not inplace)))
    if min_bytes is not None:
        attrs += ' minBytes="%d"' % min_bytes
    if max_bytes is not None:
        attrs += ' maxBytes="%d"' % max_bytes
    if nthreads is not None:
        attrs += ' nthreads="%d"' % nthreads
    o.write("<algo %s>\n" % attrs)
    for g in sorted(gpus):
        ic, oc, sc, tbs = gpus[g]
        o.write('  <gpu id="%d" i_chunks="%d" o_chunks="%d" s_chunks="%d">\n' % (g, ic, oc, sc))
        for tb in sorted(tbs, key=lambda t: t.id):
            o.write('    <tb id="%d" send="%d" recv="%d" chan="%d">\n' % (tb.id, tb.send, tb.recv, tb.chan))
            for s, (typ, sb, so, db, do, cnt, di, ds, hd) in enumerate(tb.steps):
                o.write('      <step s="%d" type="%s" srcbuf="%s" srcoff="%d" dstbuf="%s" dstoff="%d" cnt="%d" '
                        'depid="%d" deps="%d" hasdep="%d"/>\n' % (s, typ, sb, so, db, do, cnt, di, ds, hd))
            o.write("    </tb>\n")
        o.write("  </gpu>\n")
    o.write("</algo>\n")
    return o.getvalue()


def allreduce_allpairs(n: int, instances: int = 1, proto: str = "LL", inplace: bool = True,
                       min_bytes: Optional[int] = 0, max_bytes: Optional[int] = None,
                       nthreads: Optional[int] = None, name: str = "allreduce_pairs") -> str:
    """All-pairs AllReduce: reduce-scatter into scratch, local reduce, all-gather (n >= 2)."""
    if n < 2:
        raise ValueError("allpairs needs at least 2 ranks")
    I = instances
    ncpl = I * n * n
    gpus = {}
    for r in range(n):
        peers = [p for p in range(n) if p != r]
        slot = {p: i for i, p in enumerate(peers)}
        red = {k: _Tb(k, -1, -1, k) for k in range(I)}
        ptb = {}
        for pi, p in enumerate(peers):
            for k in range(I):
                tid = I + pi * I + k
                ptb[(k, p)] = _Tb(tid, p, p, k)
        ob = "i" if inplace else "o"
        # step indices that others depend on
        recv_step: Dict[Tuple[int, int], int] = {}
        red_last: Dict[Tuple[int, int], int] = {}
        copy_step: Dict[int, int] = {}
        # peer tbs, phase 1: send peer's chunks, receive peer's copy of mine into scratch
        for k in range(I):
            base = k * n * n
            for p in peers:
                tb = ptb[(k, p)]
                tb.add("s", "i", base + p * n, "s", k * (n - 1) * n + _slot_of(r, p) * n, n)
                recv_step[(k, p)] = tb.add("r", "i", base + r * n, "s", k * (n - 1) * n + slot[p] * n, n, hasdep=1)
        # reduce thread blocks (owned chunk 0 of each instance)
        for k in range(I):
            base = k * n * n
            tb = red[k]
            if not inplace:
                copy_step[k] = tb.add("cpy", "i", base + r * n, "o", base + r * n, n, hasdep=1)
            others = [ptb[(k, p)].id for p in peers]
            for dep in others[1:]:
                tb.nop(dep, 1)
            # the reduce tb reduces owned chunk j = r, peer tb (k, p) reduces owned chunk j = p
            srcs = [k * (n - 1) * n + slot[p] * n + r for p in peers]
            for i, so in enumerate(srcs):
                last = i == len(srcs) - 1
                if i == 0:
                    red_last[(k, -1)] = tb.add("re", "s", so, ob, base + r * n + r, 1, others[0], 1, int(last))
                else:
                    red_last[(k, -1)] = tb.add("re", "s", so, ob, base + r * n + r, 1, -1, -1, int(last))
        # peer tbs: reduce owned chunk j = 1 + peer index, then exchange
        for k in range(I):
            base = k * n * n
            for pi, p in enumerate(peers):
                tb = ptb[(k, p)]
                j = p
                others = [ptb[(k, q)].id for q in peers if q != p]
                first_dep = None
                if inplace:
                    for dep in others[1:]:
                        tb.nop(dep, recv_step[(k, p)])
                    if others:
                        first_dep = (others[0], recv_step[(k, p)])
                else:
                    # the reduction target o[...] is written by the reduce tb's copy
                    for dep in others:
                        tb.nop(dep, recv_step[(k, p)])
                    first_dep = (red[k].id, copy_step[k])
                srcs = [k * (n - 1) * n + slot[q] * n + j for q in peers]
                for i, so in enumerate(srcs):
                    last = i == len(srcs) - 1
                    if i == 0 and first_dep is not None:
                        idx = tb.add("re", "s", so, ob, base + r * n + j, 1, first_dep[0], first_dep[1], int(last))
                    else:
                        idx = tb.add("re", "s", so, ob, base + r * n + j, 1, -1, -1, int(last))
                red_last[(k, p)] = idx
        for k in range(I):
            base = k * n * n
            for p in peers:
                tb = ptb[(k, p)]
                for q in peers:
                    if q != p:
                        tb.nop(ptb[(k, q)].id, red_last[(k, q)])
                tb.add("s", ob, base + r * n, ob, base + r * n, n, red[k].id, red_last[(k, -1)])
                tb.add("r", ob, base + p * n, ob, base + p * n, n)
        tbs = list(red.values()) + list(ptb.values())
        gpus[r] = (ncpl, 0 if inplace else ncpl, I * (n - 1) * n, tbs)
    if max_bytes is None:
        max_bytes = SCRATCH_SCHEDULE_MAX_BYTES
    return _emit(name, proto, I, ncpl, n, "allreduce", inplace, gpus, min_bytes, max_bytes, nthreads)


def allreduce_oneshot(n: int, instances: int = 1, proto: str = "LL",
                      min_bytes: Optional[int] = 0, max_bytes: Optional[int] = None,
                      nthreads: Optional[int] = None, name: str = "allreduce_oneshot",
                      ordered: bool = False) -> str:
    """One-shot all-pairs AllReduce (in place): every rank sends its whole buffer to every peer's
    scratch, then reduces the received copies.  Fewer transfers on the critical path than the
    two-phase schedule (s, r, re instead of s, r, re, s, r), for latency-bound sizes.
    ordered=False: re folds the n-1 received copies into the rank's own buffer, d (+) s_p; for
      n == 2 and a commutative op both ranks hold the same bits, for n > 2 ranks may differ in
      floating-point rounding.
    ordered=True: rank q's data sits in scratch slot q on every rank (own data by a local cpy),
      re folds slots 1..n-1 into slot 0 and a cpy writes the result back, so every rank folds in
      rank order and all ranks hold the same bits for any n (one transfer more: s, r, re, cpy)."""
    if n < 2:
        raise ValueError("oneshot needs at least 2 ranks")
    I = instances
    nslot = n if ordered else n - 1
    gpus = {}
    for r in range(n):
        peers = [p for p in range(n) if p != r]
        red = [_Tb(k, -1, -1, k) for k in range(I)]
        ptb = {}
        for pi, p in enumerate(peers):
            for k in range(I):
                tb = _Tb(I + pi * I + k, p, p, k)
                rs = k * nslot + (p if ordered else pi)
                tb.add("s", "i", k, "s", k * nslot + (r if ordered else _slot_of(r, p)), 1)
                tb.add("r", "i", k, "s", rs, 1, hasdep=1)
                ptb[(k, p)] = tb
        for k in range(I):
            tb = red[k]
            others = [ptb[(k, p)].id for p in peers]
            if ordered:
                tb.add("cpy", "i", k, "s", k * n + r, 1)
            for dep in others[1:]:
                tb.nop(dep, 1)
            if ordered:
                for q in range(1, n):
                    if q == 1:
                        tb.add("re", "s", k * n + q, "s", k * n, 1, others[0], 1)
                    else:
                        tb.add("re", "s", k * n + q, "s", k * n, 1)
                tb.add("cpy", "s", k * n, "i", k, 1)
            else:
                for pi, p in enumerate(peers):
                    if pi == 0:
                        tb.add("re", "s", k * (n - 1) + pi, "i", k, 1, others[0], 1)
                    else:
                        tb.add("re", "s", k * (n - 1) + pi, "i", k, 1)
        tbs = red + [ptb[(k, p)] for p in peers for k in range(I)]
        gpus[r] = (I, 0, I * nslot, tbs)
    if max_bytes is None:
        max_bytes = SCRATCH_SCHEDULE_MAX_BYTES
    return _emit(name, proto, I, I, n, "allreduce", True, gpus, min_bytes, max_bytes, nthreads)


def allreduce_pair_oneshot(instances: int = 1, proto: str = "LL", inplace: bool = True,
                           min_bytes: Optional[int] = 0, max_bytes: Optional[int] = None,
                           nthreads: Optional[int] = None, name: str = "allreduce_pair_oneshot") -> str:
    """Two-rank all-pairs AllReduce in one hop: thread block k of each rank sends its chunk k to
    the peer and receives the peer's chunk k, reducing it with its own into the output (`s`,
    `rrc`).  No scratch, no cross-tb dependency: one FIFO hand-off on the critical path.  The
    reduce is fn(peer, local) (LL) on one rank and its mirror on the other, so both ranks hold
    the same bits for a commutative op."""
    I = instances
    gpus = {}
    ob = "i" if inplace else "o"
    for r in range(2):
        p = 1 - r
        tbs = []
        for k in range(I):
            tb = _Tb(k, p, p, k)
            tb.add("s", "i", k, ob, k, 1)
            tb.add("rrc", "i", k, ob, k, 1)
            tbs.append(tb)
        gpus[r] = (I, 0 if inplace else I, 0, tbs)
    if max_bytes is None:
        max_bytes = 1 << 62
    return _emit(name, proto, I, I, 2, "allreduce", inplace, gpus, min_bytes, max_bytes, nthreads)


def _slot_of(r: int, p: int) -> int:
    """scratch slot of sender r on receiver p: peers of p in ascending order, p skipped."""
    return r if r < p else r - 1


def hamiltonian_decomposition(n: int, budget: int = 200000) -> Optional[List[List[int]]]:
    """n - 1 arc-disjoint directed Hamiltonian cycles of the complete directed graph on n vertices
    (every ordered pair (i, j), i != j, is an arc of exactly one cycle), or None.  They exist for
    every n except 4 and 6 (Tillson's theorem); this is a seeded depth-first search, which finds
    them at once for the node sizes here (n = 8: the first seed, a few thousand steps).  On a fully
    connected xGMI node every GPU then sends on all n - 1 of its links when the channels' rings
    are spread over the cycles (the rotations i -> i + s with s coprime to n give only phi(n)
    of them: 4 of 7 links on 8 GPUs)."""
    import random
    if n < 2:
        return None
    if n == 2:
        return [[0, 1]]
    if n in (4, 6):
        return None
    for seed in range(64):
        rnd = random.Random(seed)
        used = [[False] * n for _ in range(n)]
        cycles: List[List[int]] = []
        steps = [0]

        def cycle(path, inpath):
            steps[0] += 1
            if steps[0] > budget:
                raise TimeoutError
            u = path[-1]
            if len(path) == n:
                if used[u][path[0]]:
                    return False
                used[u][path[0]] = True
                if solve():
                    return True
                used[u][path[0]] = False
                return False
            cand = [v for v in range(n) if not inpath[v] and not used[u][v]]
            rnd.shuffle(cand)
            for v in cand:
                used[u][v] = inpath[v] = True
                path.append(v)
                if cycle(path, inpath):
                    return True
                path.pop()
                used[u][v] = inpath[v] = False
            return False

        def solve():
            if len(cycles) == n - 1:
                return True
            path, inpath = [0], [False] * n
            inpath[0] = True
            cycles.append(path)
            if cycle(path, inpath):
                return True
            cycles.pop()
            return False
        try:
            if solve():
                return [list(c) for c in cycles]
        except TimeoutError:
            continue
    return None


def ring_cycles(n: int, channels: int) -> List[List[int]]:
    """The ring (a Hamiltonian cycle, as the rank order along it) of every channel: the n - 1
    arc-disjoint cycles of hamiltonian_decomposition dealt round-robin over the channels, or, where
    none exists (n = 4, 6), the rotations i -> i + s for s coprime to n."""
    cyc = hamiltonian_decomposition(n)
    if cyc is None:
        cyc = [[(i * s) % n for i in range(n)] for s in range(1, n) if _gcd(s, n) == 1]
    return [cyc[c % len(cyc)] for c in range(channels)]


def allreduce_ring(n: int, channels: int = 1, proto: str = "Simple", inplace: bool = True,
                   min_bytes: Optional[int] = 0, max_bytes: Optional[int] = None,
                   nthreads: Optional[int] = None, strides: Optional[List[int]] = None,
                   name: str = "allreduce_ring", rings: Optional[List[List[int]]] = None) -> str:
    """Ring AllReduce, one ring per channel: s, rrs x (n-2), rrcs, rcs x (n-2), r.

    Channel c walks rings[c] (the rank order along a Hamiltonian cycle).  Default: ring_cycles,
    the n - 1 arc-disjoint directed Hamiltonian cycles of the full mesh spread over the channels,
    so every GPU sends on all its xGMI links; `strides` gives the rotation i -> i + stride_c
    instead (the round-3 form: with strides coprime to n only phi(n) cycles exist).
    """
    if rings is None:
        if strides is not None:
            rings = [[(i * st) % n for i in range(n)] for st in strides]
        else:
            rings = ring_cycles(n, channels)
    ncpl = channels * n
    gpus = {}
    ob = "i" if inplace else "o"
    for r in range(n):
        tbs = []
        for c in range(channels):
            ring = rings[c]
            pos = ring.index(r)
            nxt = ring[(pos + 1) % n]
            prv = ring[(pos - 1) % n]
            tb = _Tb(c, nxt, prv, c)

            def ch(i):  # chunk of ring position i in channel c
                return c * n + (i % n)
            if not inplace:
                pass
            tb.add("s", "i", ch(pos), ob, ch(pos), 1)
            for t in range(1, n - 1):
                tb.add("rrs", "i", ch(pos - t), ob, ch(pos - t), 1)
            cdone = ch(pos + 1)
            tb.add("rrcs", "i", cdone, ob, cdone, 1)
            for t in range(1, n - 1):
                tb.add("rcs", ob, ch(pos + 1 - t), ob, ch(pos + 1 - t), 1)
            tb.add("r", ob, ch(pos + 2), ob, ch(pos + 2), 1)
            tbs.append(tb)
        gpus[r] = (ncpl, 0 if inplace else ncpl, 0, tbs)
    if max_bytes is None:
        max_bytes = 1 << 62
    return _emit(name, proto, channels, ncpl, n, "allreduce", inplace, gpus, min_bytes, max_bytes, nthreads)


def reduce_scatter_allpairs(n: int, instances: int = 1, proto: str = "Simple", inplace: bool = False,
                            min_bytes: Optional[int] = 0, max_bytes: Optional[int] = None,
                            nthreads: Optional[int] = None, name: str = "reduce_scatter_pairs",
                            form: str = "chain") -> str:
    """All-pairs ReduceScatter.  Input = n blocks (block q -> rank q), output = one block.

    form "chain" (default, no scratch): one thread block per (instance, peer), all links busy at
    once.  Each output chunk of instance k is cut into P pieces, P the smallest power of two >= n - 1
    (so sizes divide as the reference's power-of-two loops do).  Thread block (k, p_i) (p_i the i-th
    peer in ascending order) runs P stages; at stage t it works on piece j = (i - t) mod P: `s` of
    the piece its peer works on at stage t, then `rrc` of piece j, receiving peer p_i's copy and
    reducing it with the partial sum the piece's previous fold left in the output (a dependency on
    that thread block's stage; the first fold of a piece starts from the rank's own input block).
    Every (thread block, piece) pair meets at exactly one stage, so each piece is folded once per
    peer and every thread block is busy at every stage: the chain is pipelined over pieces.  Per
    piece the fold is ((x_r (+) x_a) (+) x_b) ... over the peers in the order their stages come,
    fn(local, peer) for Simple, fn(peer, local) for LL (oracle/sim.py runs the same program).  HBM
    bytes per output byte: 5 (n - 1), against 5 n + 1 for the scratch form.  For n = 2 it is one
    `s` + `rrc` per thread block (P = 1).
    form "scratch": every peer's copy lands in scratch (one thread block per peer) and a reduce
    thread block folds them with one fused `re` (own block first: (s0 (+) s1 ...) (+) d for Simple)."""
    I = instances
    gpus = {}
    if form == "chain":
        P = 1
        while P < n - 1:
            P *= 2
        ncpl = n * I * P
        for r in range(n):
            peers = [p for p in range(n) if p != r]
            tid = {(k, i): k * (n - 1) + i for k in range(I) for i in range(n - 1)}
            # folds of piece j: (stage, tb index) in stage order
            folds = {j: sorted(((i - j) % P, i) for i in range(n - 1)) for j in range(P)}
            tbs = []
            for k in range(I):
                for i, p in enumerate(peers):
                    tb = _Tb(tid[(k, i)], p, p, k)
                    ip = _slot_of(r, p)  # my index among p's peers
                    for t in range(P):
                        js = (ip - t) % P        # the piece of block p that p folds at stage t
                        tb.add("s", "i", p * I * P + k * P + js, "o", k * P + js, 1)
                        j = (i - t) % P
                        f = folds[j].index((t, i))
                        src = ("i", r * I * P + k * P + j) if f == 0 else ("o", k * P + j)
                        dep = (-1, -1)
                        if f > 0:
                            tp, ipv = folds[j][f - 1]
                            dep = (tid[(k, ipv)], 2 * tp + 1)
                        tb.add("rrc", src[0], src[1], "o", k * P + j, 1, dep[0], dep[1], int(f < n - 2))
                    tbs.append(tb)
            gpus[r] = (ncpl, I * P, 0, tbs)
        if max_bytes is None:
            max_bytes = 1 << 62
        return _emit(name, proto, I, ncpl, n, "reduce_scatter", inplace, gpus, min_bytes, max_bytes, nthreads)
    if form != "scratch":
        raise ValueError("form must be 'chain' or 'scratch'")
    ncpl = n * I
    if n == 2:
        for r in range(2):
            p = 1 - r
            tbs = []
            for k in range(I):
                tb = _Tb(k, p, p, k)
                tb.add("s", "i", p * I + k, "o", k, 1)
                tb.add("rrc", "i", r * I + k, "o", k, 1)
                tbs.append(tb)
            gpus[r] = (ncpl, I, 0, tbs)
        if max_bytes is None:
            max_bytes = 1 << 62
        return _emit(name, proto, I, ncpl, n, "reduce_scatter", inplace, gpus, min_bytes, max_bytes, nthreads)
    for r in range(n):
        peers = [p for p in range(n) if p != r]
        slot = {p: i for i, p in enumerate(peers)}
        tbs = []
        ptb = {}
        tid = I
        for p in peers:
            for k in range(I):
                ptb[(k, p)] = _Tb(tid, p, p, k)
                tid += 1
        recv_step = {}
        for k in range(I):
            for p in peers:
                tb = ptb[(k, p)]
                tb.add("s", "i", p * I + k, "s", k * (n - 1) + _slot_of(r, p), 1)
                recv_step[(k, p)] = tb.add("r", "i", r * I + k, "s", k * (n - 1) + slot[p], 1, hasdep=1)
        for k in range(I):
            tb = _Tb(k, -1, -1, k)
            # output chunk k starts as my own block (in-place: the output aliases input block r)
            if not inplace:
                tb.add("cpy", "i", r * I + k, "o", k, 1)
            others = [ptb[(k, p)].id for p in peers]
            for dep in others[1:]:
                tb.nop(dep, recv_step[(k, peers[0])])
            for i, p in enumerate(peers):
                last = i == len(peers) - 1
                so = k * (n - 1) + slot[p]
                if i == 0:
                    tb.add("re", "s", so, "o", k, 1, others[0], recv_step[(k, peers[0])], int(last))
                else:
                    tb.add("re", "s", so, "o", k, 1, -1, -1, int(last))
            tbs.append(tb)
        tbs += list(ptb.values())
        gpus[r] = (ncpl, I, I * (n - 1), tbs)
    if max_bytes is None:
        max_bytes = 1 << 62
    return _emit(name, proto, I, ncpl, n, "reduce_scatter", inplace, gpus, min_bytes, max_bytes, nthreads)


def allgather_allpairs(n: int, instances: int = 1, proto: str = "Simple", inplace: bool = False,
                       min_bytes: Optional[int] = 0, max_bytes: Optional[int] = None,
                       nthreads: Optional[int] = None, name: str = "allgather_pairs") -> str:
    """All-pairs AllGather.  Input = I chunks, output = n blocks of I chunks (block p from rank p)."""
    I = instances
    ncpl = n * I
    gpus = {}
    for r in range(n):
        peers = [p for p in range(n) if p != r]
        tbs = []
        tid = 0
        # out of place: the own block's copy follows the first peer's send of the same chunk, so
        # the interpreter runs the two as one copy-send (transport.cc: kSendCopy)
        for pi, p in enumerate(peers):
            for k in range(I):
                tb = _Tb(tid, p, p, k)
                tid += 1
                tb.add("s", "i", k, "o", r * I + k, 1)
                if not inplace and pi == 0:
                    tb.add("cpy", "i", k, "o", r * I + k, 1)
                tb.add("r", "i", k, "o", p * I + k, 1)
                tbs.append(tb)
        gpus[r] = (I, ncpl, 0, tbs)
    if max_bytes is None:
        max_bytes = 1 << 62
    return _emit(name, proto, I, ncpl, n, "allgather", inplace, gpus, min_bytes, max_bytes, nthreads)


def _gcd(a: int, b: int) -> int:
    while b:
        a, b = b, a % b
    return a


def write(path: str, text: str) -> str:
    with open(path, "w") as f:
        f.write(text)
    return path

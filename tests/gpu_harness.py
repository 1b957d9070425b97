"""Shared GPU parity harness: run one collective through the C-ABI on co-resident ranks and
compare with the CPU oracle (oracle/sim.py) on identical seeded inputs.

Ranks are created with ncclCommInitAll(devlist=[0]*n) so all of them live on cuda:0 and a
group of their calls is one fused launch — the same kernels, FIFOs and flag protocol as the
multi-GPU path, with local HBM in place of xGMI.
"""
from __future__ import annotations

import os
from typing import List, Optional

import numpy as np

import msccl_amd as M
from oracle import loader as L
from oracle import numerics as N
from oracle import plan as P
from oracle import sim as S

TORCH_DT = None


def torch_dtype(dt: int):
    import torch
    return {0: torch.int8, 1: torch.uint8, 2: torch.int32, 3: torch.int32, 4: torch.int64, 5: torch.int64,
            6: torch.float16, 7: torch.float32, 8: torch.float64, 9: torch.int16}[dt]


def to_torch(a: np.ndarray, dev):
    import torch
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    elif a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint16:
        a = a.view(np.int16)
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def from_torch(t, np_dtype) -> np.ndarray:
    a = t.cpu().numpy()
    return a.view(np_dtype)


def gen_inputs(n: int, count: int, dt: int, seed: int, mode: str = "uniform") -> List[np.ndarray]:
    """Per-rank inputs: uniform[-1,1) (fp) / small ints, or 'exact' small integers."""
    out = []
    for r in range(n):
        rng = np.random.default_rng(seed * 1000 + r)
        kind = N.DTYPES[dt][2]
        if kind == "int" or mode == "exact":
            v = rng.integers(-4, 5, size=count)
            if kind == "int" and N.storage(dt) in (np.uint8, np.uint32, np.uint64):
                v = rng.integers(0, 9, size=count)
            out.append(N.from_float(dt, v.astype(np.float64)) if kind != "int" else v.astype(N.storage(dt)))
        else:
            v = rng.uniform(-1.0, 1.0, size=count)
            out.append(N.from_float(dt, v))
    return out


def run_collective(xml_text: str, nranks: int, coll: int, count: int, dt: int, op: int = 0,
                   in_place: bool = True, seed: int = 1, mode: str = "uniform", iters: int = 1,
                   tmpdir: str = "/tmp", extra_xmls: Optional[List[str]] = None,
                   devices: Optional[List[int]] = None):
    """Returns (gpu_outputs, oracle_outputs) as lists of numpy arrays (interpreter element type).
    devices: the device of each rank (default: all on cuda:0, co-resident)."""
    import torch
    path = os.path.join(tmpdir, "msccl_test_%d_%d.xml" % (os.getpid(), abs(hash(xml_text)) % 100000))
    with open(path, "w") as f:
        f.write(xml_text)
    os.environ["MSCCL_XML_FILES"] = ":".join([path] + (extra_xmls or []))
    devices = list(devices) if devices is not None else [0] * nranks
    devs = [torch.device("cuda", d) for d in devices]
    comms = M.Comm.init_all(devices)
    try:
        algos = [L.parse_xml(xml_text, r, nranks) for r in range(nranks)]
        ts = N.type_size(dt)
        if coll == L.ALLREDUCE:
            in_n, out_n = count, count
        elif coll == L.REDUCE_SCATTER:
            in_n, out_n = count * nranks, count
        else:  # allgather
            in_n, out_n = count, count * nranks
        ins = gen_inputs(nranks, in_n, dt, seed, mode)
        # GPU
        t_in = [to_torch(x, devs[r]) for r, x in enumerate(ins)]
        if in_place:
            if coll == L.ALLREDUCE:
                t_out = t_in
                sends = [t.data_ptr() for t in t_in]
                recvs = sends
            elif coll == L.REDUCE_SCATTER:
                t_out = [t[r * count:(r + 1) * count] for r, t in enumerate(t_in)]
                sends = [t.data_ptr() for t in t_in]
                recvs = [t.data_ptr() for t in t_out]
            else:
                t_out = [torch.zeros(out_n, dtype=t_in[0].dtype, device=devs[r]) for r in range(nranks)]
                for r in range(nranks):
                    t_out[r][r * count:(r + 1) * count] = t_in[r]
                sends = [t_out[r][r * count:(r + 1) * count].data_ptr() for r in range(nranks)]
                recvs = [t.data_ptr() for t in t_out]
        else:
            t_out = [torch.full((out_n,), 7, dtype=t_in[0].dtype, device=devs[r]) for r in range(nranks)]
            sends = [t.data_ptr() for t in t_in]
            recvs = [t.data_ptr() for t in t_out]
        for d in set(devs):
            torch.cuda.synchronize(d)
        streams = [torch.cuda.current_stream(d).cuda_stream for d in devs]
        for _ in range(iters):
            with M.group():
                for r, c in enumerate(comms):
                    if coll == L.ALLREDUCE:
                        c.all_reduce(sends[r], recvs[r], count, dt, op, streams[r])
                    elif coll == L.REDUCE_SCATTER:
                        c.reduce_scatter(sends[r], recvs[r], count, dt, op, streams[r])
                    else:
                        c.all_gather(sends[r], recvs[r], count, dt, streams[r])
        for d in set(devs):
            torch.cuda.synchronize(d)
        for c in comms:
            err = c.async_error()
            if err != 0:
                raise M.NcclError(err, "kernel (async error)")
        gpu = [from_torch(t, N.storage(dt) if coll != L.ALLGATHER else N.storage(dt)) for t in t_out]
        run_collective.last = [c.info()["last"] for c in comms]  # the kernel each rank's last launch took
    finally:
        for c in comms:
            c.destroy()
    # oracle
    call = P.Call(coll, count, dt, op, nranks, 0, in_place)
    idx = P.select([algos[0]], call)
    assert idx == 0, "oracle selection failed"
    plan = P.make_plan([algos[0]], call, 0)
    o_in = [x.copy() for x in ins]
    if coll == L.ALLGATHER:
        o_in = [x.view(np.int8) for x in o_in]
        o_out = [np.zeros(out_n * ts, np.int8) for _ in range(nranks)]
    elif in_place:
        o_out = [None] * nranks
    else:
        o_out = [np.full(out_n, 7, N.storage(dt)) if N.DTYPES[dt][2] != "bf16" else np.full(out_n, 7, np.uint16)
                 for _ in range(nranks)]
    for _ in range(iters):
        res, _ = S.run(algos, plan, o_in, o_out, coll, in_place)
        if iters > 1 and coll == L.ALLREDUCE and in_place:
            o_in = res
    if coll == L.ALLGATHER:
        res = [r.view(N.storage(dt)) for r in res]
    return gpu, [np.asarray(r) for r in res], ins


def run_ring_fallback(nranks: int, coll: int, count: int, dt: int, op: int = 0, in_place: bool = True,
                      seed: int = 1, mode: str = "uniform", iters: int = 1, user_scale=None):
    """No MSCCL schedule loaded: every call takes the ring fallback (enqueue.cc:461-476).
    op 4 = ncclAvg.  user_scale=(value, residence): each rank creates a PreMulSum op with that
    scale (residence 1 host immediate, 0 device scalar) and uses it.
    Returns (gpu_outputs, oracle_outputs, ring_params) compared by the caller."""
    import torch
    from oracle import ring as R
    os.environ.pop("MSCCL_XML_FILES", None)
    os.environ.pop("MSCCL_CONFIG", None)
    dev = torch.device("cuda:0")
    comms = M.Comm.init_all([0] * nranks)
    ops = [op] * nranks
    dev_op, arg = op, 0
    if op == N.AVG:
        dev_op, arg = N.avg_op(dt, nranks)
    scale_dev = None
    if user_scale is not None:
        value, residence = user_scale
        dev_op, arg = N.PREMULSUM, N.scalar_bits(dt, value)
        sb = int(arg).to_bytes(8, "little")[:N.type_size(dt)]
        if residence == 0:
            scale_dev = torch.frombuffer(bytearray(sb), dtype=torch.uint8).to(dev)
            torch.cuda.synchronize()
        ops = [c.create_premulsum(sb if residence == 1 else scale_dev.data_ptr(), dt, residence) for c in comms]
    try:
        if coll == L.ALLREDUCE:
            in_n, out_n = count, count
        elif coll == L.REDUCE_SCATTER:
            in_n, out_n = count * nranks, count
        else:
            in_n, out_n = count, count * nranks
        ins = gen_inputs(nranks, in_n, dt, seed, mode)
        t_in = [to_torch(x, dev) for x in ins]
        if in_place:
            if coll == L.ALLREDUCE:
                t_out, sends, recvs = t_in, [t.data_ptr() for t in t_in], [t.data_ptr() for t in t_in]
            elif coll == L.REDUCE_SCATTER:
                t_out = [t[r * count:(r + 1) * count] for r, t in enumerate(t_in)]
                sends, recvs = [t.data_ptr() for t in t_in], [t.data_ptr() for t in t_out]
            else:
                t_out = [torch.zeros(out_n, dtype=t_in[0].dtype, device=dev) for _ in range(nranks)]
                for r in range(nranks):
                    t_out[r][r * count:(r + 1) * count] = t_in[r]
                sends = [t_out[r][r * count:(r + 1) * count].data_ptr() for r in range(nranks)]
                recvs = [t.data_ptr() for t in t_out]
        else:
            t_out = [torch.full((out_n,), 7, dtype=t_in[0].dtype, device=dev) for _ in range(nranks)]
            sends, recvs = [t.data_ptr() for t in t_in], [t.data_ptr() for t in t_out]
        torch.cuda.synchronize()
        stream = torch.cuda.current_stream().cuda_stream
        for _ in range(iters):
            with M.group():
                for r, c in enumerate(comms):
                    if coll == L.ALLREDUCE:
                        c.all_reduce(sends[r], recvs[r], count, dt, ops[r], stream)
                    elif coll == L.REDUCE_SCATTER:
                        c.reduce_scatter(sends[r], recvs[r], count, dt, ops[r], stream)
                    else:
                        c.all_gather(sends[r], recvs[r], count, dt, stream)
        torch.cuda.synchronize()
        for c in comms:
            if c.async_error() != 0:
                raise M.NcclError(c.async_error(), "kernel (async error)")
        gpu = [from_torch(t, N.storage(dt)) for t in t_out]
        last = comms[0].info()["last"]   # what the product ran (ringColl 4 chain tree, 5 flat tree)
        if user_scale is not None:
            for c, o in zip(comms, ops):
                c.destroy_op(o)
    finally:
        for c in comms:
            c.destroy()
    o_in = [x.copy() for x in ins]
    if coll == L.ALLGATHER:
        o_out = [np.zeros(out_n, N.storage(dt)) for _ in range(nranks)]
    elif in_place:
        o_out = [None] * nranks
    else:
        o_out = [np.full(out_n, 7, N.storage(dt)) for _ in range(nranks)]
    res = None
    for _ in range(iters):
        res, rp = R.run(coll, count, dt, dev_op, o_in, o_out, in_place, arg)
        if iters > 1 and coll == L.ALLREDUCE and in_place:
            o_in = res
    rp = dict(rp, last=last)
    return gpu, [np.asarray(r) for r in res], rp


# ---------------------------------------------------------------------------------------------
# Mismatch reports and numeric bounds shared by the parity tests


def describe_mismatch(got: np.ndarray, want: np.ndarray, chunk_elems: Optional[int] = None, limit: int = 6) -> str:
    """Where two arrays differ: count, first runs of differing elements (with their MSCCL chunk
    when chunk_elems is given) and whether the bad values are zeros or equal to other places of
    the expected array (misplaced data) — enough to localise a FIFO or offset fault from one
    failure record."""
    g = np.ascontiguousarray(got).view(np.uint8).reshape(len(got), -1)
    w = np.ascontiguousarray(want).view(np.uint8).reshape(len(want), -1)
    bad = np.flatnonzero((g != w).any(axis=1))
    if len(bad) == 0:
        return "identical"
    runs = np.split(bad, np.flatnonzero(np.diff(bad) != 1) + 1)
    out = ["%d of %d elements differ in %d runs" % (len(bad), len(got), len(runs))]
    for run in runs[:limit]:
        a, b = int(run[0]), int(run[-1]) + 1
        seg = g[a:b]
        what = "zeros" if not seg.any() else "values"
        where = ""
        if chunk_elems:
            where = " (chunk %d +%d)" % (a // chunk_elems, a % chunk_elems)
        out.append("  [%d, %d)%s: %s, got %s want %s" % (a, b, where, what, got[a:min(b, a + 3)], want[a:min(b, a + 3)]))
    return "\n".join(out)


def sum_error_ok(result: np.ndarray, inputs: List[np.ndarray], dt: int) -> tuple:
    """Checks |result - exact sum| <= (n-1) * u * sum|x_i| elementwise (the classical bound for
    any association order of n-1 roundings at unit roundoff u), and returns (ok, worst ratio)."""
    n = len(inputs)
    u = {6: 2.0 ** -11, 7: 2.0 ** -24, 9: 2.0 ** -8, 8: 2.0 ** -53}[dt]
    xs = [N.to_float64(dt, x) for x in inputs]
    exact = np.sum(xs, axis=0)
    mag = np.sum(np.abs(xs), axis=0)
    err = np.abs(N.to_float64(dt, result) - exact)
    bound = (n - 1) * u * mag + 1e-30
    ratio = float(np.max(err / bound)) if len(err) else 0.0
    return ratio <= 1.0, ratio


class CoResident:
    """n ranks on cuda:0 created by one ncclCommInitAll with several XML schedules registered
    (MSCCL_XML_FILES, as a user registers size tiers).  run() issues one grouped collective;
    oracle() computes what the reference would produce for the same call: the schedule the
    reference's selection picks (oracle/plan.py), or its ring fallback (oracle/ring.py)."""

    def __init__(self, n: int, xml_texts: List[str], tmpdir: str = "/tmp"):
        self.n = n
        self.paths = []
        for i, x in enumerate(xml_texts):
            p = os.path.join(tmpdir, "msccl_cores_%d_%d_%d.xml" % (os.getpid(), i, abs(hash(x)) % 100000))
            with open(p, "w") as f:
                f.write(x)
            self.paths.append(p)
        os.environ["MSCCL_XML_FILES"] = ":".join(self.paths)
        self.algos = [[L.parse_xml(x, r, n) for x in xml_texts] for r in range(n)]
        self.comms = M.Comm.init_all([0] * n)

    def close(self):
        for c in self.comms:
            c.destroy()
        self.comms = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def run(self, coll: int, count: int, dt: int, op: int, sends, recvs, stream: int = 0):
        import torch
        with M.group():
            for r, c in enumerate(self.comms):
                if coll == L.ALLREDUCE:
                    c.all_reduce(sends[r], recvs[r], count, dt, op, stream)
                elif coll == L.REDUCE_SCATTER:
                    c.reduce_scatter(sends[r], recvs[r], count, dt, op, stream)
                else:
                    c.all_gather(sends[r], recvs[r], count, dt, stream)
        torch.cuda.synchronize()
        for c in self.comms:
            if c.async_error() != 0:
                raise M.NcclError(c.async_error(), "kernel (async error)")

    def oracle(self, coll: int, count: int, dt: int, op: int, ins: List[np.ndarray], in_place: bool):
        """Expected outputs (interpreter element type) and the schedule used ('ring' or index)."""
        call = P.Call(coll, count, dt, op, self.n, 0, in_place)
        idx = P.select(self.algos[0], call)
        ts = N.type_size(dt)
        out_n = count if coll != L.ALLGATHER else count * self.n
        if idx is None:
            from oracle import ring as R
            o_in = [x.copy() for x in ins]
            o_out = [None] * self.n if in_place and coll == L.ALLREDUCE else \
                [np.zeros(out_n, N.storage(dt)) for _ in range(self.n)]
            res, _ = R.run(coll, count, dt, op, o_in, o_out, in_place)
            return [np.asarray(r) for r in res], "ring"
        algos = [a[idx] for a in self.algos]
        plan = P.make_plan(self.algos[0], call, idx)
        o_in = [x.copy() for x in ins]
        if coll == L.ALLGATHER:
            o_in = [x.view(np.int8) for x in o_in]
            o_out = [np.zeros(out_n * ts, np.int8) for _ in range(self.n)]
        elif in_place:
            o_out = [None] * self.n
        else:
            o_out = [np.zeros(out_n, N.storage(dt)) for _ in range(self.n)]
        res, _ = S.run(algos, plan, o_in, o_out, coll, in_place)
        res = [np.asarray(r) for r in res]
        if coll == L.ALLGATHER:
            res = [r.view(N.storage(dt)) for r in res]
        return res, idx

#!/usr/bin/env python3
"""Small-message latency decomposition: HIP-event time per launch (2 co-resident ranks, 128 B per
rank) for schedules that add one ingredient at a time (a local copy, more copies, a cross-tb
dependency flag, a send/recv pair, the all-pairs AllReduce).  Also prints the device trace span
of the last launch when MSCCL_AMD_TRACE=1.
  python tools/latency_probe.py [--bytes 128] [--iters 200]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import msccl_amd as M  # noqa: E402
from msccl_amd import xmlgen as X  # noqa: E402


def ag_xml(name, build, proto="LL"):
    """2-rank AllGather-typed schedule (i_chunks 1, o_chunks 2); build(r, tbs) adds the tbs."""
    gpus = {}
    for r in range(2):
        tbs = []
        build(r, tbs)
        gpus[r] = (1, 2, 0, tbs)
    return X._emit(name, proto, 1, 2, 2, "allgather", False, gpus, 0, 1 << 62)


def cpy(k):
    def b(r, tbs):
        tb = X._Tb(0, -1, -1, 0)
        for _ in range(k):
            tb.add("cpy", "i", 0, "o", r, 1)
        tbs.append(tb)
    return b


def cpy_dep(r, tbs):
    t0 = X._Tb(0, -1, -1, 0)
    t0.add("cpy", "i", 0, "o", r, 1, hasdep=1)
    t1 = X._Tb(1, -1, -1, 0)
    t1.add("cpy", "i", 0, "o", r, 1, depid=0, deps=0)
    tbs += [t0, t1]


def send_recv(r, tbs):
    p = 1 - r
    tb = X._Tb(0, p, p, 0)
    tb.add("s", "i", 0, "o", r, 1)
    tb.add("r", "i", 0, "o", p, 1)
    tbs.append(tb)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=128)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--proto", default="LL")
    ap.add_argument("--case", type=int, default=-1, help="run only this case (index)")
    a = ap.parse_args()
    import torch
    cases = [
        ("cpy x1", ag_xml("p1", cpy(1), a.proto), M.Comm.all_gather),
        ("cpy x4", ag_xml("p4", cpy(4), a.proto), M.Comm.all_gather),
        ("cpy -> flag -> cpy", ag_xml("pd", cpy_dep, a.proto), M.Comm.all_gather),
        ("s, r", ag_xml("psr", send_recv, a.proto), M.Comm.all_gather),
        ("allpairs AllReduce", X.allreduce_allpairs(2, 1, a.proto), M.Comm.all_reduce),
    ]
    cnt = a.bytes // 4
    if a.case >= 0:
        cases = cases[a.case:a.case + 1]
    for name, xml, fn in cases:
        path = "/tmp/lat_probe_%d.xml" % os.getpid()
        open(path, "w").write(xml)
        os.environ["MSCCL_XML_FILES"] = path
        comms = M.Comm.init_all([0, 0])
        ins = [torch.ones(cnt * 2, device="cuda") for _ in comms]
        outs = [torch.zeros(cnt * 2, device="cuda") for _ in comms]

        def step():
            with M.group():
                for c, i, o in zip(comms, ins, outs):
                    if fn is M.Comm.all_reduce:
                        c.all_reduce(i.data_ptr(), i.data_ptr(), cnt, M.FLOAT32, M.SUM, 0)
                    else:
                        c.all_gather(i.data_ptr(), o.data_ptr(), cnt, M.FLOAT32, 0)
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            step()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / a.iters
        print("%-22s %7.2f us per launch" % (name, us), flush=True)
        for c in comms:
            c.destroy()


if __name__ == "__main__":
    main()

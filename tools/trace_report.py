#!/usr/bin/env python3
"""Latency breakdown of one MSCCL launch from the device event trace (MSCCL_AMD_TRACE=1).

  python tools/trace_report.py [--bytes N] [--proto LL] [--ranks 2] [--instances 1]

Runs a few grouped AllReduces of the all-pairs schedule on co-resident ranks of cuda:0, then
prints, per workgroup slot of the last launch, the time (us, from the earliest workgroup start)
of each event: setup, dependency waits, primitive begin/end.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MSCCL_AMD_TRACE", "1")  # 2: small kernel kept (start, end + XCD)
import msccl_amd as M  # noqa: E402
from msccl_amd import xmlgen  # noqa: E402

TT = {0: "s", 1: "r", 2: "rcs", 3: "rrs", 4: "rrc", 5: "rrcs", 6: "cpy", 7: "re"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=128)
    ap.add_argument("--proto", default="LL")
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--instances", type=int, default=1)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--schedule", default="allpairs", choices=["allpairs", "pair", "ring", "oneshot"])
    a = ap.parse_args()
    import torch
    path = "/tmp/trace_ap_%d.xml" % os.getpid()
    gen = {"allpairs": lambda: xmlgen.allreduce_allpairs(a.ranks, a.instances, a.proto),
           "pair": lambda: xmlgen.allreduce_pair_oneshot(a.instances, a.proto),
           "ring": lambda: xmlgen.allreduce_ring(a.ranks, a.instances, a.proto),
           "oneshot": lambda: xmlgen.allreduce_oneshot(a.ranks, a.instances, a.proto, ordered=a.ranks > 2)}
    open(path, "w").write(gen[a.schedule]())
    os.environ["MSCCL_XML_FILES"] = path
    comms = M.Comm.init_all([0] * a.ranks)
    cnt = a.bytes // 4
    bufs = [torch.ones(cnt, device="cuda") for _ in comms]
    for _ in range(a.iters):
        with M.group():
            for c, b in zip(comms, bufs):
                c.all_reduce(b.data_ptr(), b.data_ptr(), cnt, M.FLOAT32, M.SUM, 0)
    torch.cuda.synchronize()
    traces = [np.asarray(c.trace()) for c in comms]
    t0 = min(int(tr[s, 0]["ts"]) for tr in traces for s in range(tr.shape[0]) if tr[s, 0]["type"] == 0xFFFF)
    for r, tr in enumerate(traces):
        for s in range(tr.shape[0]):
            h = tr[s, 0]
            if h["type"] != 0xFFFF:
                continue
            parts = ["start %.2f" % ((int(h["ts"]) - t0) / 100.0)]
            for e in tr[s, 1:int(h["step"])]:
                t = (int(e["ts"]) - t0) / 100.0
                name = M.TRACE_TYPES.get(int(e["type"]), "?")
                if name == "begin":
                    parts.append("%s#%d[%s %d] %.2f" % (name, e["step"], TT.get(int(e["arg"]) >> 24, "?"),
                                                         int(e["arg"]) & 0xFFFFFF, t))
                elif name in ("dep", "end"):
                    parts.append("%s#%d %.2f" % (name, e["step"], t))
                elif name == "done" and os.environ.get("MSCCL_AMD_TRACE") == "2":
                    parts.append("done %.2f xcc %d" % (t, int(e["arg"])))
                else:
                    parts.append("%s %.2f" % (name, t))
            print("rank %d slot %3d: %s" % (r, s, " | ".join(parts)))
    for c in comms:
        c.destroy()


if __name__ == "__main__":
    main()

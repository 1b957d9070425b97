#!/usr/bin/env python3
"""Median per-event timeline over all workgroups of the last launch (device trace).
  python tools/trace_summary.py --bytes N --instances I [--proto LL]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["MSCCL_AMD_TRACE"] = "1"
import msccl_amd as M  # noqa: E402
from msccl_amd import xmlgen  # noqa: E402

TT = {0: "s", 1: "r", 2: "rcs", 3: "rrs", 4: "rrc", 5: "rrcs", 6: "cpy", 7: "re"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=1 << 20)
    ap.add_argument("--proto", default="LL")
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--instances", type=int, default=16)
    a = ap.parse_args()
    import torch
    path = "/tmp/trace_sum_%d.xml" % os.getpid()
    open(path, "w").write(xmlgen.allreduce_allpairs(a.ranks, a.instances, a.proto))
    os.environ["MSCCL_XML_FILES"] = path
    comms = M.Comm.init_all([0] * a.ranks)
    cnt = a.bytes // 4
    bufs = [torch.ones(cnt, device="cuda") for _ in comms]
    for _ in range(6):
        with M.group():
            for c, b in zip(comms, bufs):
                c.all_reduce(b.data_ptr(), b.data_ptr(), cnt, M.FLOAT32, M.SUM, 0)
    torch.cuda.synchronize()
    traces = [np.asarray(c.trace()) for c in comms]
    t0 = min(int(tr[s, 0]["ts"]) for tr in traces for s in range(tr.shape[0]) if tr[s, 0]["type"] == 0xFFFF)
    t1 = 0
    rows = {}
    for tr in traces:
        for s in range(tr.shape[0]):
            h = tr[s, 0]
            if h["type"] != 0xFFFF:
                continue
            evs = tr[s, 1:int(h["step"])]
            key = tuple((int(e["type"]), int(e["step"])) for e in evs)
            rows.setdefault(key, []).append([(int(h["ts"]) - t0) / 100.0] + [(int(e["ts"]) - t0) / 100.0 for e in evs])
            t1 = max(t1, (int(evs[-1]["ts"]) - t0) / 100.0)
    print("launch span %.2f us, %d workgroup shapes" % (t1, len(rows)))
    for key, vals in rows.items():
        v = np.median(np.array(vals), axis=0)
        names = ["start"] + ["%s%d" % (M.TRACE_TYPES.get(t, "?"), st) for t, st in key]
        print("%d wgs: " % len(vals) + " ".join("%s=%.2f" % (n, x) for n, x in zip(names, v)))
    for c in comms:
        c.destroy()


if __name__ == "__main__":
    main()

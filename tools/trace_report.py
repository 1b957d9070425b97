#!/usr/bin/env python3
"""Where one MSCCL launch spends its time, from the device event trace (MSCCL_AMD_TRACE=1).

  python tools/trace_report.py [--schedule allpairs|pair|ring|oneshot] [--bytes N] [--proto LL]
                               [--ranks 2] [--instances 1] [--dtype 7] [--summary]

Runs a few grouped AllReduces of the schedule on co-resident ranks of cuda:0, then prints, per
workgroup slot of the last launch, the time (us, from the earliest workgroup start) of each event:
setup, dependency waits, primitive begin/end.  --summary instead aggregates over every workgroup
per transfer index: mean and max duration of the primitive call, and of it the time the polling
lane waited for the Simple tail (data from the previous rank) and for send credit (the next rank
freeing a FIFO slot), plus the gaps between calls: a launch's time split into streaming and
stalls.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MSCCL_AMD_TRACE", "1")  # 2: small kernel kept (start, end + XCD)
import msccl_amd as M  # noqa: E402
from msccl_amd import xmlgen  # noqa: E402

TT = {0: "s", 1: "r", 2: "rcs", 3: "rrs", 4: "rrc", 5: "rrcs", 6: "cpy", 7: "re", 9: "copysend", 10: "s+rrc",
      11: "s+cpy"}


def summarize(traces):
    """Per transfer index over every workgroup: duration, tail / credit waits, gap since the
    previous event of the workgroup (us)."""
    t0 = min(int(tr[s, 0]["ts"]) for tr in traces for s in range(tr.shape[0]) if tr[s, 0]["type"] == 0xFFFF)
    rows = {}
    ends = []
    for tr in traces:
        for s in range(tr.shape[0]):
            h = tr[s, 0]
            if h["type"] != 0xFFFF:
                continue
            prev = int(h["ts"])
            begin = None
            for e in tr[s, 1:int(h["step"])]:
                name = M.TRACE_TYPES.get(int(e["type"]), "?")
                ts = int(e["ts"])
                if name == "begin":
                    begin = (ts, int(e["step"]), TT.get(int(e["arg"]) >> 24, "?"), ts - prev)
                elif name == "end" and begin is not None:
                    b_ts, idx, typ, gap = begin
                    r = rows.setdefault(idx, {"type": typ, "dur": [], "tail": [], "head": [], "gap": []})
                    r["dur"].append((ts - b_ts) / 100.0)
                    r["tail"].append((int(e["arg"]) >> 16) / 100.0)
                    r["head"].append((int(e["arg"]) & 0xFFFF) / 100.0)
                    r["gap"].append(gap / 100.0)
                    begin = None
                elif name == "done":
                    ends.append((ts - t0) / 100.0)
                prev = ts
    out = []
    tot = {"dur": 0.0, "tail": 0.0, "head": 0.0, "gap": 0.0}
    for idx in sorted(rows):
        r = rows[idx]
        m = {k: float(np.mean(r[k])) for k in ("dur", "tail", "head", "gap")}
        for k in tot:
            tot[k] += m[k]
        out.append("transfer %2d %-6s  call %7.2f us (max %7.2f)  tail wait %7.2f  credit wait %7.2f  gap before %5.2f"
                   % (idx, r["type"], m["dur"], max(r["dur"]), m["tail"], m["head"], m["gap"]))
    out.append("sum of means: calls %.1f us = tail waits %.1f + credit waits %.1f + moving %.1f; gaps %.1f; "
               "launch end (slowest workgroup) %.1f us, median %.1f"
               % (tot["dur"], tot["tail"], tot["head"], tot["dur"] - tot["tail"] - tot["head"], tot["gap"],
                  max(ends) if ends else 0, float(np.median(ends)) if ends else 0))
    return out


def by_tb(traces, max_split):
    """Per thread block (slot // maxSplit), mean over its workgroups and ranks: time in primitive
    calls, time outside them (dependency waits, flag publishes, setup), and when it ended (us from
    the earliest start): which thread blocks the launch waits for."""
    t0 = min(int(tr[s, 0]["ts"]) for tr in traces for s in range(tr.shape[0]) if tr[s, 0]["type"] == 0xFFFF)
    rows = {}
    for tr in traces:
        for s in range(tr.shape[0]):
            h = tr[s, 0]
            if h["type"] != 0xFFFF:
                continue
            start = prev = int(h["ts"])
            calls = 0
            types = []
            begin = None
            end = prev
            for e in tr[s, 1:int(h["step"])]:
                name = M.TRACE_TYPES.get(int(e["type"]), "?")
                ts = int(e["ts"])
                if name == "begin":
                    begin = ts
                    t = TT.get(int(e["arg"]) >> 24, "?")
                    if not types or types[-1] != t:
                        types.append(t)
                elif name == "end" and begin is not None:
                    calls += ts - begin
                    begin = None
                end = ts
            r = rows.setdefault(s // max_split, {"calls": [], "other": [], "end": [], "types": types})
            r["calls"].append(calls / 100.0)
            r["other"].append((end - start - calls) / 100.0)
            r["end"].append((end - t0) / 100.0)
    out = []
    for tb in sorted(rows):
        r = rows[tb]
        out.append("tb %3d %-28s calls %8.1f us  outside calls %8.1f  end %8.1f (max %8.1f)  [%d wgs]"
                   % (tb, ",".join(r["types"][:6]), np.mean(r["calls"]), np.mean(r["other"]), np.mean(r["end"]),
                      max(r["end"]), len(r["end"])))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=128)
    ap.add_argument("--proto", default="LL")
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--instances", type=int, default=1)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--dtype", type=int, default=7, help="ncclDataType_t: 7 fp32, 6 fp16, 9 bf16")
    ap.add_argument("--schedule", default="allpairs",
                    choices=["allpairs", "pair", "ring", "oneshot", "allgather", "reducescatter", "rccl32"])
    ap.add_argument("--summary", action="store_true")
    ap.add_argument("--by-tb", action="store_true", help="per thread block: busy, outside calls, end")
    a = ap.parse_args()
    import torch
    path = "/tmp/trace_ap_%d.xml" % os.getpid()
    big = 1 << 40
    gen = {"allpairs": lambda: xmlgen.allreduce_allpairs(a.ranks, a.instances, a.proto, max_bytes=big),
           "pair": lambda: xmlgen.allreduce_pair_oneshot(a.instances, a.proto),
           "ring": lambda: xmlgen.allreduce_ring(a.ranks, a.instances, a.proto),
           "oneshot": lambda: xmlgen.allreduce_oneshot(a.ranks, a.instances, a.proto, ordered=a.ranks > 2),
           # C5's pair (bench.py run_extra): --bytes is the whole buffer, a rank's block is bytes / ranks
           "allgather": lambda: xmlgen.allgather_allpairs(a.ranks, a.instances, a.proto, False, 0, big),
           "reducescatter": lambda: xmlgen.reduce_scatter_allpairs(a.ranks, a.instances, a.proto, False, 0, big,
                                                                   form="chain"),
           # RCCL's shipped 8-rank all-pairs LL file, maxBytes raised (bench.py secondary_schedules)
           "rccl32": lambda: open("/opt/rocm/share/rccl/msccl-algorithms/allreduce-allpairs-8n-ll-32tb.xml").read()
           .replace('maxBytes="65536"', 'maxBytes="%d"' % big)}
    open(path, "w").write(gen[a.schedule]())
    os.environ["MSCCL_XML_FILES"] = path
    comms = M.Comm.init_all([0] * a.ranks)
    ts = {7: 4, 6: 2, 9: 2}[a.dtype]
    cnt = a.bytes // ts
    bufs = [torch.zeros((a.bytes + 3) // 4, device="cuda") for _ in comms]
    outs = [torch.zeros((a.bytes + 3) // 4, device="cuda") for _ in comms]
    blk = cnt // a.ranks
    for _ in range(a.iters):
        with M.group():
            for c, b, o in zip(comms, bufs, outs):
                if a.schedule == "allgather":
                    c.all_gather(b.data_ptr(), o.data_ptr(), blk, a.dtype, 0)
                elif a.schedule == "reducescatter":
                    c.reduce_scatter(b.data_ptr(), o.data_ptr(), blk, a.dtype, M.SUM, 0)
                else:
                    c.all_reduce(b.data_ptr(), b.data_ptr(), cnt, a.dtype, M.SUM, 0)
    torch.cuda.synchronize()
    traces = [np.asarray(c.trace()) for c in comms]
    if a.by_tb:
        print("%s x%d, %d ranks, %d B per rank, %s, dtype %d, per thread block:" % (
            a.schedule, a.instances, a.ranks, a.bytes, a.proto, a.dtype))
        for line in by_tb(traces, comms[0].info()["maxSplit"]):
            print(line)
    elif a.summary:
        print("%s x%d, %d ranks, %d B per rank, %s, dtype %d:" % (a.schedule, a.instances, a.ranks, a.bytes,
                                                                 a.proto, a.dtype))
        for line in summarize(traces):
            print(line)
    else:
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
                    elif name == "end":
                        parts.append("end#%d %.2f (waits tail %.2f credit %.2f)" % (
                            e["step"], t, (int(e["arg"]) >> 16) / 100.0, (int(e["arg"]) & 0xFFFF) / 100.0))
                    elif name == "dep":
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

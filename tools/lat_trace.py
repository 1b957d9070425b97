"""Where the device time of one small fused pair launch goes (a MSCCL_LAT_TRACE build of the
library: tools/lat/libmsccl_amd_lat.so, MSCCL_AMD_TRACE=2).  Runs back-to-back 2-rank pair
AllReduces and prints, per trace point, the median time (us) from the workgroup's start:
  10 prologue done, 11 fused op entry, 12 first step's lines sent, 13 peer lines received and
  output stored, 14 head posted, 15 pass done, 16 epilogue done;
then, over every workgroup of a launch, how far apart the workgroups started and ended (us).
  MSCCL_AMD_LIB=tools/lat/libmsccl_amd_lat.so MSCCL_AMD_TRACE=2 python tools/lat_trace.py [bytes] [instances]
With LAT_TRACE_SCHEDULE=allpairs the pair kernel's points (PairRunner: 10 prologue done, 11-14 in
the fused op, 15 op done, 16 epilogue done) of a lowered 2-rank all-pairs call (> 4 KiB)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import msccl_amd as M  # noqa: E402
from msccl_amd import xmlgen  # noqa: E402


def main():
    import torch
    nbytes = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    inst = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    path = "/tmp/lat_trace_%d.xml" % os.getpid()
    # LAT_TRACE_SCHEDULE=allpairs: the msccl-tools two-phase all-pairs (bench.py's C2 tiers), whose
    # calls above 4 KiB run lowered on the pair kernel (PairRunner's trace points, same ids)
    if os.environ.get("LAT_TRACE_SCHEDULE", "pair") == "allpairs":
        open(path, "w").write(xmlgen.allreduce_allpairs(2, inst, "LL"))
    else:
        open(path, "w").write(xmlgen.allreduce_pair_oneshot(inst, "LL"))
    os.environ["MSCCL_XML_FILES"] = path
    comms = M.Comm.init_all([0, 0])
    cnt = nbytes // 4
    bufs = [torch.ones(cnt, device="cuda") for _ in comms]
    rows = {}
    spread = {"start": [], "end": [], "rank1_later": []}
    stream = torch.cuda.Stream()

    def step():
        with M.group():
            for c, b in zip(comms, bufs):
                c.all_reduce(b.data_ptr(), b.data_ptr(), cnt, M.FLOAT32, M.SUM, stream.cuda_stream)
    graph = None
    if os.environ.get("LAT_TRACE_GRAPH", "1") == "1":
        # steady state: each sample is the last launch of a replayed graph of 20 back-to-back launches
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream, capture_error_mode="relaxed"):
            for _ in range(20):
                step()
        torch.cuda.synchronize()
    for it in range(300):
        if graph is not None:
            with torch.cuda.stream(stream):
                graph.replay()
        else:
            step()
        if it < 20:
            continue
        torch.cuda.synchronize()
        starts, ends, first = [], [], {}
        for r, c in enumerate(comms):
            tr = np.asarray(c.trace())
            for s in range(tr.shape[0]):
                h = tr[s, 0]
                if h["type"] != 0xFFFF:
                    continue
                t0 = int(h["ts"])
                starts.append(t0)
                first.setdefault(r, t0)
                evs = tr[s, 1:int(h["step"])]
                if len(evs):
                    ends.append(int(evs[-1]["ts"]))
                if s == 0:
                    for e in evs:
                        rows.setdefault((r, int(e["type"])), []).append((int(e["ts"]) - t0) / 100.0)
        if starts:
            spread["start"].append((max(starts) - min(starts)) / 100.0)
            spread["end"].append((max(ends) - min(starts)) / 100.0 if ends else 0)
        if len(first) == 2:
            spread["rank1_later"].append((first[1] - first[0]) / 100.0)
    for (r, t) in sorted(rows):
        v = np.array(rows[(r, t)])
        print("rank %d point %d: median %.2f us (p10 %.2f, p90 %.2f, n %d)" % (
            r, t, np.median(v), np.percentile(v, 10), np.percentile(v, 90), len(v)))
    for k, v in spread.items():
        if v:
            print("%s: median %.2f us (p10 %.2f, p90 %.2f)" % (
                {"start": "workgroup starts span", "end": "first start to last trace point",
                 "rank1_later": "rank 1 slot 0 starts after rank 0 slot 0 by"}[k],
                np.median(v), np.percentile(v, 10), np.percentile(v, 90)))
    for c in comms:
        c.destroy()


if __name__ == "__main__":
    main()

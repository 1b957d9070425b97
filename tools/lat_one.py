"""Back-to-back launches of one small AllReduce (for rocprofv3 kernel durations / HIP events).
  python tools/lat_one.py [--schedule pair|allpairs|oneshot|ring] [--bytes 128] [--ranks 2] [--instances 1]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import msccl_amd as M  # noqa: E402
from msccl_amd import xmlgen  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--schedule", default="pair")
    ap.add_argument("--bytes", type=int, default=128)
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--instances", type=int, default=1)
    ap.add_argument("--proto", default="LL")
    ap.add_argument("--dtype", type=int, default=7)
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--coll", default="ar", choices=["ar", "rs", "ag"],
                    help="AllReduce, or ReduceScatter / AllGather with --bytes per rank's block "
                         "(agap / rsap, or the fallback: fbring there is the ring, fbtree the flat form)")
    ap.add_argument("--graph", action="store_true",
                    help="capture the launches in one hipGraph and time its replay: device time per launch "
                         "without the host's per-call cost")
    a = ap.parse_args()
    import torch
    gen = {"allpairs": lambda: xmlgen.allreduce_allpairs(a.ranks, a.instances, a.proto),
           "pair": lambda: xmlgen.allreduce_pair_oneshot(a.instances, a.proto),
           "ring": lambda: xmlgen.allreduce_ring(a.ranks, a.instances, a.proto),
           "oneshot": lambda: xmlgen.allreduce_oneshot(a.ranks, a.instances, a.proto, ordered=a.ranks > 2),
           # C5's pair (--coll ag / rs, --bytes a rank's block)
           "agap": lambda: xmlgen.allgather_allpairs(a.ranks, a.instances, a.proto, False, 0, 1 << 40),
           "rsap": lambda: xmlgen.reduce_scatter_allpairs(a.ranks, a.instances, a.proto, False, 0, 1 << 40,
                                                          form="chain"),
           # RCCL's shipped 8-rank all-pairs LL file, maxBytes raised (bench.py secondary_schedules)
           "rccl32": lambda: open("/opt/rocm/share/rccl/msccl-algorithms/allreduce-allpairs-8n-ll-32tb.xml").read()
           .replace('maxBytes="65536"', 'maxBytes="%d"' % (1 << 40))}
    if a.schedule == "empty":
        # the floor: a one-element torch kernel per launch, captured and replayed the same way
        x = torch.zeros(1, device="cuda")
        stream = torch.cuda.Stream()
        with torch.cuda.stream(stream):
            for _ in range(20):
                x.add_(1)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for _ in range(a.iters):
                x.add_(1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        with torch.cuda.stream(stream):
            g.replay()
        e1.record(stream)
        torch.cuda.synchronize()
        print("empty (one-element add) kernel: %.2f us per launch (events, graph replay)"
              % (e0.elapsed_time(e1) * 1000 / a.iters), flush=True)
        return
    if a.schedule in ("fbring", "fbtree", "fbchain"):   # no schedule: the ring / tree fallback
        os.environ.pop("MSCCL_XML_FILES", None)
        os.environ["NCCL_ALGO"] = "Ring" if a.schedule == "fbring" else "Tree"
        if a.schedule == "fbchain":   # the chain tree (fbtree: the flat tree where it applies)
            os.environ["MSCCL_AMD_TREE_FLAT"] = "0"
        if a.coll != "ar":           # the ring, or (fbtree) its flat form
            os.environ["NCCL_ALGO"] = "Ring,Tree"
            if a.schedule == "fbring":
                os.environ["MSCCL_AMD_TREE_FLAT"] = "0"
    else:
        path = "/tmp/lat_one_%d.xml" % os.getpid()
        open(path, "w").write(gen[a.schedule]())
        os.environ["MSCCL_XML_FILES"] = path
    comms = M.Comm.init_all([0] * a.ranks)
    ts = {7: 4, 6: 2, 9: 2}[a.dtype]
    cnt = a.bytes // ts
    bufs = [torch.ones(cnt * ts // 4 + 1, device="cuda") for _ in comms]
    big = [torch.ones(cnt * a.ranks * ts // 4 + 1, device="cuda") for _ in comms] if a.coll != "ar" else None

    stream = torch.cuda.Stream()

    def step():
        with M.group():
            for i, (c, b) in enumerate(zip(comms, bufs)):
                if a.coll == "ar":
                    c.all_reduce(b.data_ptr(), b.data_ptr(), cnt, a.dtype, M.SUM, stream.cuda_stream)
                elif a.coll == "rs":
                    c.reduce_scatter(big[i].data_ptr(), b.data_ptr(), cnt, a.dtype, M.SUM, stream.cuda_stream)
                else:
                    c.all_gather(b.data_ptr(), big[i].data_ptr(), cnt, a.dtype, stream.cuda_stream)
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    import time
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    graph = None
    if a.graph:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream, capture_error_mode="relaxed"):
            for _ in range(a.iters):
                step()
        torch.cuda.synchronize()
    e0.record(stream)
    t0 = time.perf_counter()
    if graph is not None:
        with torch.cuda.stream(stream):
            graph.replay()
    else:
        for _ in range(a.iters):
            step()
    host = (time.perf_counter() - t0) / a.iters
    e1.record(stream)
    torch.cuda.synchronize()
    last = comms[0].info()["last"]
    print("%s%s %d B x%d ranks: %.2f us per launch (events%s), host %.2f us per call; ran ringColl %d small %d pair %d" % (
        a.schedule, "" if a.coll == "ar" else "-" + a.coll, a.bytes, a.ranks, e0.elapsed_time(e1) * 1000 / a.iters, ", graph replay" if graph else "",
        host * 1e6, last["ringColl"], last["small"], last.get("pair", 0)), flush=True)
    for c in comms:
        c.destroy()


if __name__ == "__main__":
    main()

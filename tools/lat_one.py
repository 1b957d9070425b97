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
    a = ap.parse_args()
    import torch
    gen = {"allpairs": lambda: xmlgen.allreduce_allpairs(a.ranks, a.instances, a.proto),
           "pair": lambda: xmlgen.allreduce_pair_oneshot(a.instances, a.proto),
           "ring": lambda: xmlgen.allreduce_ring(a.ranks, a.instances, a.proto),
           "oneshot": lambda: xmlgen.allreduce_oneshot(a.ranks, a.instances, a.proto, ordered=a.ranks > 2)}
    if a.schedule in ("fbring", "fbtree"):   # no schedule: the ring / tree fallback
        os.environ.pop("MSCCL_XML_FILES", None)
        os.environ["NCCL_ALGO"] = "Ring" if a.schedule == "fbring" else "Tree"
    else:
        path = "/tmp/lat_one_%d.xml" % os.getpid()
        open(path, "w").write(gen[a.schedule]())
        os.environ["MSCCL_XML_FILES"] = path
    comms = M.Comm.init_all([0] * a.ranks)
    ts = {7: 4, 6: 2, 9: 2}[a.dtype]
    cnt = a.bytes // ts
    bufs = [torch.ones(cnt * ts // 4 + 1, device="cuda") for _ in comms]

    def step():
        with M.group():
            for c, b in zip(comms, bufs):
                c.all_reduce(b.data_ptr(), b.data_ptr(), cnt, a.dtype, M.SUM, 0)
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    import time
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        step()
    host = (time.perf_counter() - t0) / a.iters
    e1.record()
    torch.cuda.synchronize()
    print("%s %d B x%d ranks: %.2f us per launch (events), host %.2f us per call" % (
        a.schedule, a.bytes, a.ranks, e0.elapsed_time(e1) * 1000 / a.iters, host * 1e6), flush=True)
    for c in comms:
        c.destroy()


if __name__ == "__main__":
    main()

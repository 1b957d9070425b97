"""Where the device time of one small fused pair launch goes (a MSCCL_LAT_TRACE build of the
library: tools/ab/libmsccl_amd_lat.so, MSCCL_AMD_TRACE=2).  Runs back-to-back 2-rank 128 B pair
AllReduces and prints, per trace point, the median time (us) from the workgroup's start:
  10 prologue done, 11 fused op entry, 12 first step's lines sent, 13 peer lines received and
  output stored, 14 head posted, 15 pass done, 16 epilogue done.
  MSCCL_AMD_LIB=tools/ab/libmsccl_amd_lat.so MSCCL_AMD_TRACE=2 python tools/lat_trace.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import msccl_amd as M  # noqa: E402
from msccl_amd import xmlgen  # noqa: E402


def main():
    import torch
    nbytes = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    path = "/tmp/lat_trace_%d.xml" % os.getpid()
    open(path, "w").write(xmlgen.allreduce_pair_oneshot(1, "LL"))
    os.environ["MSCCL_XML_FILES"] = path
    comms = M.Comm.init_all([0, 0])
    cnt = nbytes // 4
    bufs = [torch.ones(cnt, device="cuda") for _ in comms]
    rows = {}
    for it in range(300):
        with M.group():
            for c, b in zip(comms, bufs):
                c.all_reduce(b.data_ptr(), b.data_ptr(), cnt, M.FLOAT32, M.SUM, 0)
        if it < 20:
            continue
        torch.cuda.synchronize()
        for r, c in enumerate(comms):
            tr = np.asarray(c.trace())
            h = tr[0, 0]
            if h["type"] != 0xFFFF:
                continue
            t0 = int(h["ts"])
            for e in tr[0, 1:int(h["step"])]:
                rows.setdefault((r, int(e["type"])), []).append((int(e["ts"]) - t0) / 100.0)
    for (r, t) in sorted(rows):
        v = np.array(rows[(r, t)])
        print("rank %d point %d: median %.2f us (p10 %.2f, p90 %.2f, n %d)" % (
            r, t, np.median(v), np.percentile(v, 10), np.percentile(v, 90), len(v)))
    for c in comms:
        c.destroy()


if __name__ == "__main__":
    main()

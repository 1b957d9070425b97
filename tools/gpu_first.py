"""First-contact GPU check: a few collectives on co-resident ranks vs the oracle."""
import os, sys, time, traceback
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "10")
import numpy as np
import torch
from tests.gpu_harness import run_collective
from msccl_amd import xmlgen
from oracle import loader as L
cases = [
  ("ap2 LL f32 1k", xmlgen.allreduce_allpairs(2, 1, "LL"), 2, L.ALLREDUCE, 1024, 7, True),
  ("ap2 LL f32 1M", xmlgen.allreduce_allpairs(2, 4, "LL"), 2, L.ALLREDUCE, 1 << 18, 7, True),
  ("ap2 Simple f32 1M", xmlgen.allreduce_allpairs(2, 4, "Simple"), 2, L.ALLREDUCE, 1 << 18, 7, True),
  ("ap8 LL f16 64k", xmlgen.allreduce_allpairs(8, 4, "LL"), 8, L.ALLREDUCE, 1 << 15, 6, True),
  ("ring8 Simple bf16", xmlgen.allreduce_ring(8, 4, "Simple"), 8, L.ALLREDUCE, 1 << 18, 9, True),
  ("rs8 Simple f32", xmlgen.reduce_scatter_allpairs(8, 2, "Simple"), 8, L.REDUCE_SCATTER, 1 << 14, 7, False),
  ("ag8 Simple f32", xmlgen.allgather_allpairs(8, 2, "Simple"), 8, L.ALLGATHER, 1 << 14, 7, False),
]
ok = True
for name, x, n, coll, cnt, dt, ip in cases:
    t = time.time()
    try:
        g, o, _ = run_collective(x, n, coll, cnt, dt, 0, ip)
        bad = [r for r in range(n) if not np.array_equal(g[r].view(np.uint8), o[r].view(np.uint8))]
        print("%-22s %s  %.2fs  bad ranks %s" % (name, "OK " if not bad else "FAIL", time.time() - t, bad), flush=True)
        if bad:
            r = bad[0]; d = np.nonzero(g[r].view(np.uint8) != o[r].view(np.uint8))[0]
            print("   first diff byte", d[:10], "of", len(d), flush=True)
            ok = False
    except Exception as e:
        traceback.print_exc()
        print("%-22s ERROR %s" % (name, e), flush=True)
        ok = False
        break
sys.exit(0 if ok else 1)

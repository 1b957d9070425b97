"""Print GPU vs oracle vs inputs around the first failing element of one case."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "10")
from msccl_amd import xmlgen  # noqa: E402
from oracle import loader as L  # noqa: E402
from tests.gpu_harness import run_collective, gen_inputs  # noqa: E402

for proto in ("Simple", "LL"):
    os.environ["MSCCL_AMD_SPLIT"] = "1"
    x = xmlgen.allreduce_allpairs(2, 1, proto)
    n, count = 2, 4 * 1024
    gpu, ora, ins = run_collective(x, n, L.ALLREDUCE, count, 7, mode="exact")
    g, o = gpu[0], np.asarray(ora[0])
    bad = np.nonzero(g != o)[0]
    print(proto, "bad", len(bad), "of", count, "runs:", [(int(a), int(b)) for a, b in zip(bad[:-1], bad[1:]) if b != a + 1][:10])
    for e in [0, 255, 256, 257, 1024, 2047, 2048, 2303, 2304, 4095]:
        print("  e=%d in0=%g in1=%g gpu=%g ora=%g" % (e, ins[0][e], ins[1][e], g[e], o[e]))

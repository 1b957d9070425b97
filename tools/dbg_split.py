"""Isolate split/merge/unroll parity failures on one GPU: run a case under several knob settings."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "10")
from msccl_amd import xmlgen  # noqa: E402
from oracle import loader as L  # noqa: E402
from tests.gpu_harness import run_collective  # noqa: E402


def one(tag, env, xml, n, count, dt):
    for k in ("MSCCL_AMD_SPLIT", "MSCCL_AMD_MERGE"):
        os.environ.pop(k, None)
    os.environ.update(env)
    try:
        gpu, ora, _ = run_collective(xml, n, L.ALLREDUCE, count, dt)
    except Exception as e:  # noqa: BLE001
        print(tag, env, "ERROR", e, flush=True)
        return
    msgs = []
    for r in range(n):
        g, o = gpu[r], np.asarray(ora[r])
        bad = np.nonzero(g.view(np.uint8).reshape(len(g), -1).any(axis=1) != 0) if False else None
        diff = np.nonzero(g.view(np.uint32 if g.itemsize == 4 else np.uint16) != o.view(np.uint32 if o.itemsize == 4 else np.uint16))[0]
        if len(diff):
            msgs.append("r%d: %d bad elems, first %s" % (r, len(diff), diff[:6].tolist()))
    print(tag, env, "OK" if not msgs else "FAIL " + "; ".join(msgs), flush=True)


for proto in ("LL", "Simple"):
    x = xmlgen.allreduce_allpairs(2, 4, proto)
    for env in ({}, {"MSCCL_AMD_MERGE": "1"}, {"MSCCL_AMD_SPLIT": "1"}, {"MSCCL_AMD_SPLIT": "2"},
                {"MSCCL_AMD_SPLIT": "2", "MSCCL_AMD_MERGE": "1"}, {"MSCCL_AMD_SPLIT": "8", "MSCCL_AMD_MERGE": "1"}):
        one(proto + " 262144", env, x, 2, 262144, 7)
    one(proto + " 1<<16 single-iter", {}, x, 2, 1 << 16, 7)
    one(proto + " 1<<16 single-iter split1", {"MSCCL_AMD_SPLIT": "1"}, x, 2, 1 << 16, 7)

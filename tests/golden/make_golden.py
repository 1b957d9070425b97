"""Generate the golden input/output vectors in tests/golden/ from the CPU oracle (oracle/sim.py).

The reference ships no test vectors for this path, so these fixtures
are produced by the oracle and committed: they pin the oracle against regressions and give the
GPU tests fixed expected outputs.  Exact-integer cases are additionally self-checking (any
association order gives the same bits).  Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from msccl_amd import xmlgen  # noqa: E402
from oracle import loader as L  # noqa: E402
from oracle import numerics as N  # noqa: E402
from oracle import plan as P  # noqa: E402
from oracle import sim as S  # noqa: E402

RCCL = "/opt/rocm/share/rccl/msccl-algorithms"

CASES = [
    # name, xml-text-or-path, nranks, coll, count, dtype, op, inplace, mode
    ("ap2_ll_f32", lambda: xmlgen.allreduce_allpairs(2, 4, "LL"), 2, L.ALLREDUCE, 4096, 7, 0, True, "uniform"),
    ("ap2_simple_f32_small", lambda: xmlgen.allreduce_allpairs(2, 1, "Simple"), 2, L.ALLREDUCE, 1000, 7, 0, True, "uniform"),
    ("ap4_ll_bf16", lambda: xmlgen.allreduce_allpairs(4, 2, "LL"), 4, L.ALLREDUCE, 2048, 9, 0, True, "uniform"),
    ("ap8_ll_f16_rccl32tb", lambda: open(os.path.join(RCCL, "allreduce-allpairs-8n-ll-32tb.xml")).read(), 8,
     L.ALLREDUCE, 8192, 6, 0, True, "uniform"),
    ("ap8_simple_f32_op", lambda: xmlgen.allreduce_allpairs(8, 1, "Simple", inplace=False), 8, L.ALLREDUCE, 4096,
     7, 0, False, "uniform"),
    # the rotation rings of round 3 (strides 1, 3, 5, 7), pinned: the default rings are now the
    # Hamiltonian decomposition (xmlgen.ring_cycles), whose association order differs
    ("ring8_simple_bf16", lambda: xmlgen.allreduce_ring(8, 4, "Simple", strides=[1, 3, 5, 7]), 8, L.ALLREDUCE, 4096, 9, 0, True, "uniform"),
    ("ring4_ll_f32_max", lambda: xmlgen.allreduce_ring(4, 2, "LL"), 4, L.ALLREDUCE, 800, 7, 2, True, "uniform"),
    ("rs8_simple_f32", lambda: xmlgen.reduce_scatter_allpairs(8, 2, "Simple", form="scratch"), 8, L.REDUCE_SCATTER, 512, 7, 0,
     False, "uniform"),
    ("ag8_ll_f32", lambda: xmlgen.allgather_allpairs(8, 2, "LL"), 8, L.ALLGATHER, 512, 7, 0, False, "uniform"),
    ("ap2_ll_i32_exact", lambda: xmlgen.allreduce_allpairs(2, 2, "LL"), 2, L.ALLREDUCE, 1024, 2, 0, True, "exact"),
    ("ap4_ll128_f16", lambda: xmlgen.allreduce_allpairs(4, 2, "LL128"), 4, L.ALLREDUCE, 32 * 1001, 6, 0, True,
     "uniform"),
]

# Ring fallback (no schedule matches, oracle/ring.py): name, nranks, coll, count, dtype, op, inplace
RING_CASES = [
    ("fb3_ring_ar_f32", 3, L.ALLREDUCE, 5003, 7, 0, True),
    ("fb4_ring_rs_bf16", 4, L.REDUCE_SCATTER, 3001, 9, 0, False),
    ("fb2_ring_ag_f16", 2, L.ALLGATHER, 777, 6, 0, False),
    ("fb8_ring_ar_f16_max", 8, L.ALLREDUCE, 100003, 6, 2, False),
]


def gen_inputs(n, count, dt, seed, mode):
    out = []
    for r in range(n):
        rng = np.random.default_rng(seed * 1000 + r)
        if N.DTYPES[dt][2] == "int" or mode == "exact":
            v = rng.integers(-4, 5, size=count)
            out.append(v.astype(N.storage(dt)) if N.DTYPES[dt][2] == "int" else N.from_float(dt, v.astype(np.float64)))
        else:
            out.append(N.from_float(dt, rng.uniform(-1.0, 1.0, size=count)))
    return out


def run_case(xml, n, coll, count, dt, op, inplace, mode, seed=7):
    algos = [L.parse_xml(xml, r, n) for r in range(n)]
    call = P.Call(coll, count, dt, op, n, 0, inplace)
    idx = P.select([algos[0]], call)
    assert idx == 0
    plan = P.make_plan([algos[0]], call, 0)
    in_n = count * n if coll == L.REDUCE_SCATTER else count
    ins = gen_inputs(n, in_n, dt, seed, mode)
    ts = N.type_size(dt)
    if coll == L.ALLGATHER:
        o_in = [x.view(np.int8).copy() for x in ins]
        outs = [np.zeros(count * n * ts, np.int8) for _ in range(n)]
    elif inplace:
        o_in = [x.copy() for x in ins]
        outs = [None] * n
    else:
        o_in = [x.copy() for x in ins]
        outs = [np.zeros(count, ins[0].dtype) for _ in range(n)]
    res, _ = S.run(algos, plan, o_in, outs, coll, inplace)
    if coll == L.ALLGATHER:
        res = [r.view(ins[0].dtype) for r in res]
    return ins, [np.array(r) for r in res]


def run_ring_case(n, coll, count, dt, op, inplace, seed=7):
    """The RING_CASES fixtures are ring fallback outputs (small AllReduces would take the tree by
    default, oracle/ring.py): the ring is pinned."""
    from oracle import ring as R
    os.environ["NCCL_ALGO"] = "Ring,Tree"
    os.environ["MSCCL_AMD_TREE_MAX_BYTES"] = "0"
    in_n = count * n if coll == L.REDUCE_SCATTER else count
    ins = gen_inputs(n, in_n, dt, seed, "uniform")
    if coll == L.ALLGATHER:
        outs = [np.zeros(count * n, ins[0].dtype) for _ in range(n)]
    elif inplace:
        outs = [None] * n
    else:
        outs = [np.zeros(count, ins[0].dtype) for _ in range(n)]
    res, _ = R.run(coll, count, dt, op, [x.copy() for x in ins], outs, inplace)
    return ins, [np.array(r) for r in res]


def main():
    for (name, n, coll, count, dt, op, inplace) in RING_CASES:
        ins, outs = run_ring_case(n, coll, count, dt, op, inplace)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), inputs=np.stack(ins), outputs=np.stack(outs),
                            meta=np.array([n, coll, count, dt, op, int(inplace)], dtype=np.int64))
        print("wrote", name)
    for (name, xf, n, coll, count, dt, op, inplace, mode) in CASES:
        xml = xf()
        ins, outs = run_case(xml, n, coll, count, dt, op, inplace, mode)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), inputs=np.stack(ins), outputs=np.stack(outs),
                            meta=np.array([n, coll, count, dt, op, int(inplace)], dtype=np.int64))
        print("wrote", name)


if __name__ == "__main__":
    main()

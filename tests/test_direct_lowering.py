"""The direct form of Simple schedules, on the host (lower.cc: analyzeDirectLowering, no GPU).

A Simple AllGather / ReduceScatter / AllReduce schedule has a direct form when its dataflow,
followed symbolically with the reference's Simple semantics (`re` = (s_0 (+) s_1 ...) (+) d,
prims_simple.h:258-263; rrs / rrc fn(local, peer)), gives the AllGather's definition, a left fold
of every rank's block per ReduceScatter output chunk, or one fold per AllReduce chunk held by every
rank.  The orders the analysis reports are checked against oracle/sim.py running the XML on float
inputs (test_direct_orders_match_the_simulator), so the analysis is not only checked against itself."""
import os

import numpy as np
import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from oracle import loader as L

RCCL = "/opt/rocm/share/rccl/msccl-algorithms"


def _write(tmp_path, xml, name="s.xml"):
    p = tmp_path / name
    p.write_text(xml)
    return str(p)


def test_c5_pair_has_direct_forms(tmp_path):
    for n in (2, 4, 8):
        rs = M.direct_json(_write(tmp_path, xmlgen.reduce_scatter_allpairs(n, 2, "Simple", False)), n)
        assert rs["ok"] == 1 and rs["coll"] == L.REDUCE_SCATTER, rs
        ag = M.direct_json(_write(tmp_path, xmlgen.allgather_allpairs(n, 2, "Simple", False)), n)
        assert ag["ok"] == 1 and ag["coll"] == L.ALLGATHER, ag
        # the scratch form of the ReduceScatter too
        rs2 = M.direct_json(_write(tmp_path, xmlgen.reduce_scatter_allpairs(n, 1, "Simple", False, form="scratch")), n)
        assert rs2["ok"] == 1, rs2


def test_ring_and_allpairs_allreduce_direct(tmp_path):
    ring = M.direct_json(_write(tmp_path, xmlgen.allreduce_ring(8, 4, "Simple", True)), 8)
    assert ring["ok"] == 1 and ring["coll"] == L.ALLREDUCE, ring
    # a ring folds each chunk along its ring from the rank after its owner: one order per (ring,
    # start), 4 rings over different Hamiltonian cycles x 8 starts
    assert len(ring["classes"]) == 32, ring
    ap = M.direct_json(_write(tmp_path, xmlgen.allreduce_allpairs(4, 2, "Simple")), 4)
    assert ap["ok"] == 1, ap


def test_rccl_simple_allpairs_direct(tmp_path):
    p = os.path.join(RCCL, "allreduce-allpairs-8n-simple.xml")
    if not os.path.exists(p):
        pytest.skip("fixture missing")
    d = M.direct_json(p, 8)
    assert d["ok"] == 1 and d["coll"] == L.ALLREDUCE, d


@pytest.mark.parametrize("xml,n,why", [
    (lambda: xmlgen.allreduce_allpairs(4, 1, "LL"), 4, "protocol is not Simple"),
    (lambda: xmlgen.allgather_allpairs(4, 1, "Simple", True), 4, "in-place"),
    (lambda: xmlgen.allreduce_oneshot(4, 4, "Simple"), 4, "different folds"),
])
def test_no_direct_form(tmp_path, xml, n, why):
    d = M.direct_json(_write(tmp_path, xml()), n)
    assert d["ok"] == 0 and why in d["why"], d


@pytest.mark.parametrize("maker,n,coll", [
    (lambda: xmlgen.allreduce_ring(4, 2, "Simple", True), 4, L.ALLREDUCE),
    (lambda: xmlgen.allreduce_allpairs(3, 1, "Simple"), 3, L.ALLREDUCE),
    (lambda: xmlgen.reduce_scatter_allpairs(4, 1, "Simple", False), 4, L.REDUCE_SCATTER),
    (lambda: xmlgen.reduce_scatter_allpairs(3, 2, "Simple", False, form="scratch"), 3, L.REDUCE_SCATTER),
])
def test_direct_orders_match_the_simulator(tmp_path, maker, n, coll):
    """The direct form's per-chunk fold orders reproduce oracle/sim.py's float results bit for bit:
    fold every rank's chunk in the analysis' order (fp32, values chosen so the order matters) and
    compare with the simulator running the XML (Simple, large-call path)."""
    from oracle import numerics as N
    from oracle import plan as P
    from oracle import sim as S
    xml = maker()
    d = M.direct_json(_write(tmp_path, xml), n)
    assert d["ok"] == 1, d
    algos = [L.parse_xml(xml, r, n) for r in range(n)]
    cnt_chunk = 1024                                        # >= nthreads (544): the large-call path
    ncpl = M.algo_json(_write(tmp_path, xml, "a.xml"), 0, n)["nchunksperloop"]
    count = (ncpl // n if coll == L.REDUCE_SCATTER else ncpl) * cnt_chunk
    in_n = count * n if coll == L.REDUCE_SCATTER else count
    rng = np.random.default_rng(5)
    ins = [(rng.standard_normal(in_n) * 10.0 ** rng.integers(-3, 4, in_n)).astype(np.float32) for _ in range(n)]
    call = P.Call(coll, count, 7, 0, n, 0, coll == L.ALLREDUCE)
    plan = P.make_plan([algos[0]], call, 0)
    outs = [None] * n if coll == L.ALLREDUCE else [np.zeros(count, np.float32) for _ in range(n)]
    res, _ = S.run(algos, plan, [x.copy() for x in ins], outs, coll, coll == L.ALLREDUCE)
    nchunks_out = count // cnt_chunk
    for r in range(n):
        got = np.asarray(res[r]).view(np.float32)
        for c in range(nchunks_out):
            order = d["classes"][d["chunkClass"][c]][r]
            base = (r * count if coll == L.REDUCE_SCATTER else 0) + c * cnt_chunk
            acc = ins[order[0]][base:base + cnt_chunk].copy()
            for q in order[1:]:
                acc = (acc + ins[q][base:base + cnt_chunk]).astype(np.float32)
            assert np.array_equal(acc.view(np.uint32), got[c * cnt_chunk:(c + 1) * cnt_chunk].view(np.uint32)), (r, c, order)

"""One-hop MSCCL AllReduce schedules run as the fold kernel (msccl_amd/csrc/lower.cc).

The product decides symbolically, from every rank's program, whether a schedule's result is on
every rank, chunk by chunk, a left fold of all ranks' same chunk (chunks grouped into classes of
equal orders); this file pins that decision against the oracle: for every schedule the product
lowers, oracle/sim.py (the reference's interpreter semantics, msccl_interpreter.h:66-205) running
the XML gives bit for bit, chunk by chunk, the fold in the product's order for that chunk's class,
on fp16 sums whose rounding depends on the order; schedules whose result is not such a fold are
refused with the reason.  No GPU needed."""
import os

import numpy as np
import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from oracle import loader as L
from oracle import numerics as N
from oracle import plan as P
from oracle import sim as S
from tests.gpu_harness import gen_inputs

RCCL = "/opt/rocm/share/rccl/msccl-algorithms"

LOWERED = {
    "pair_x1": (lambda: xmlgen.allreduce_pair_oneshot(1, "LL"), 2),
    "pair_x16": (lambda: xmlgen.allreduce_pair_oneshot(16, "LL"), 2),
    "pair_out_of_place": (lambda: xmlgen.allreduce_pair_oneshot(4, "LL", inplace=False), 2),
    "oneshot_ordered_8": (lambda: xmlgen.allreduce_oneshot(8, 4, "LL", ordered=True), 8),
    "oneshot_unordered_8": (lambda: xmlgen.allreduce_oneshot(8, 2, "LL"), 8),
    "oneshot_unordered_3": (lambda: xmlgen.allreduce_oneshot(3, 1, "LL"), 3),
    "oneshot_ordered_16": (lambda: xmlgen.allreduce_oneshot(16, 1, "LL", ordered=True), 16),
    "allpairs_2": (lambda: xmlgen.allreduce_allpairs(2, 4, "LL"), 2),
    # the two-phase all-pairs: each chunk's owner folds it first (one class per owner order)
    "allpairs_8": (lambda: xmlgen.allreduce_allpairs(8, 1, "LL"), 8),
    "allpairs_4_out_of_place": (lambda: xmlgen.allreduce_allpairs(4, 2, "LL", inplace=False), 4),
    # rings: one class per (ring, start rank) of the reduce-scatter leg
    "ring_8x1": (lambda: xmlgen.allreduce_ring(8, 1, "LL"), 8),
    "ring_8x2": (lambda: xmlgen.allreduce_ring(8, 2, "LL"), 8),
    "rccl_allpairs_8n_ll_32tb": (lambda: open(os.path.join(RCCL, "allreduce-allpairs-8n-ll-32tb.xml")).read(), 8),
}
REFUSED = {
    "ring_8x4": (lambda: xmlgen.allreduce_ring(8, 4, "LL"), 8, "more fold orders"),   # 32 orders
    "pair_simple": (lambda: xmlgen.allreduce_pair_oneshot(1, "Simple"), 2, "not LL"),
    "oneshot_ll128": (lambda: xmlgen.allreduce_oneshot(4, 1, "LL128"), 4, "not LL"),
    "reduce_scatter": (lambda: xmlgen.reduce_scatter_allpairs(4, 1, "LL"), 4, "not a valid AllReduce"),
    "allgather": (lambda: xmlgen.allgather_allpairs(4, 1, "LL"), 4, "not a valid AllReduce"),
}


def _path(tmp_path, name, text):
    p = tmp_path / (name + ".xml")
    p.write_text(text)
    return str(p)


def _oracle_run(xml, n, count, dt, in_place, seed):
    algos = [L.parse_xml(xml, r, n) for r in range(n)]
    call = P.Call(L.ALLREDUCE, count, dt, 0, n, 0, in_place)
    plan = P.make_plan([algos[0]], call, 0)
    ins = gen_inputs(n, count, dt, seed)
    outs = [None] * n if in_place else [np.zeros(count, N.storage(dt)) for _ in range(n)]
    res, _ = S.run(algos, plan, [x.copy() for x in ins], outs, L.ALLREDUCE, in_place)
    return ins, [np.asarray(r) for r in res]


def _fold(ins, order, dt):
    acc = ins[order[0]].copy()
    for q in order[1:]:
        acc = N.apply(0, dt, acc, ins[q])
    return acc


@pytest.mark.parametrize("name", sorted(LOWERED))
def test_lowered_schedules_equal_the_fold_in_their_order(tmp_path, name):
    gen, n = LOWERED[name]
    try:
        xml = gen()
    except OSError:
        pytest.skip("fixture missing")
    info = M.lower_json(_path(tmp_path, name, xml), n)
    assert info["ok"] == 1, info
    classes, cls = info["classes"], info["chunkClass"]
    assert all(len(k) == n and all(sorted(o) == list(range(n)) for o in k) for k in classes)
    a0 = L.parse_xml(xml, 0, n)
    assert len(cls) == a0.nchunksperloop and set(cls) == set(range(len(classes)))
    per = 96                            # fp16 sums of 96-element chunks: rounding depends on the order
    count = a0.nchunksperloop * per
    for dt, seed in ((6, 3), (9, 4), (7, 5)):
        ins, res = _oracle_run(xml, n, count, dt, bool(a0.inplace), seed)
        for r in range(n):
            for c in range(a0.nchunksperloop):
                sl = slice(c * per, (c + 1) * per)
                want = _fold([x[sl] for x in ins], classes[cls[c]][r], dt)
                assert np.array_equal(res[r][sl].view(np.uint8), want.view(np.uint8)), (name, dt, r, c)


def test_order_is_sensitive():
    """The check above would catch a wrong order: the unordered one-shot's ranks fold in
    different orders, and on fp16 inputs those give different bits."""
    xml = xmlgen.allreduce_oneshot(8, 1, "LL")
    ins, res = _oracle_run(xml, 8, 64 * 96, 6, True, 7)
    assert not np.array_equal(res[0].view(np.uint16), res[3].view(np.uint16))
    assert not np.array_equal(_fold(ins, list(range(8)), 6).view(np.uint16),
                              _fold(ins, [0, 3, 1, 2, 4, 5, 6, 7], 6).view(np.uint16))


def test_expected_orders(tmp_path):
    pair = M.lower_json(_path(tmp_path, "p", xmlgen.allreduce_pair_oneshot(2, "LL")), 2)
    assert pair["classes"] == [[[0, 1], [0, 1]]] and pair["chunkClass"] == [0, 0]
    ordered = M.lower_json(_path(tmp_path, "o", xmlgen.allreduce_oneshot(8, 4, "LL", ordered=True)), 8)
    assert ordered["classes"] == [[list(range(8))] * 8]
    unordered = M.lower_json(_path(tmp_path, "u", xmlgen.allreduce_oneshot(4, 1, "LL")), 4)
    # rank r: d = x_r first, then the peers ascending (fn(x_r, x_p0) is the innermost pair)
    assert unordered["classes"] == [[[0, 1, 2, 3], [0, 1, 2, 3], [0, 2, 1, 3], [0, 3, 1, 2]]]
    # the two-phase all-pairs, 4 ranks: chunk j*4+m of an instance is owned by rank j, which folds
    # it first; owners 0 and 1 give the same order (fn(x_0, x_1) either way): 3 classes
    ap = M.lower_json(_path(tmp_path, "a", xmlgen.allreduce_allpairs(4, 1, "LL")), 4)
    assert ap["chunkClass"] == [0] * 8 + [1] * 4 + [2] * 4
    assert ap["classes"] == [[[0, 1, 2, 3]] * 4, [[0, 2, 1, 3]] * 4, [[0, 3, 1, 2]] * 4]


@pytest.mark.parametrize("name", sorted(REFUSED))
def test_refused_schedules(tmp_path, name):
    gen, n, why = REFUSED[name]
    info = M.lower_json(_path(tmp_path, name, gen()), n)
    assert info["ok"] == 0 and why in info["why"], info


def test_rccl_shipped_allpairs_lowers_with_one_class_per_owner_order():
    """msccl-tools' two-phase all-pairs (RCCL's 8n 32-tb file): the owner of each chunk folds it
    first, so chunks fall into 7 classes (owners 0 and 1 fold alike)."""
    p = os.path.join(RCCL, "allreduce-allpairs-8n-ll-32tb.xml")
    if not os.path.exists(p):
        pytest.skip("fixture missing")
    info = M.lower_json(p, 8)
    assert info["ok"] == 1 and len(info["classes"]) == 7 and len(info["chunkClass"]) == 256, info


def test_broken_schedule_is_refused(tmp_path):
    """A receive that no peer sends to: the symbolic run does not complete."""
    xml = xmlgen.allreduce_pair_oneshot(1, "LL").replace('type="s"', 'type="nop"', 1)
    info = M.lower_json(_path(tmp_path, "broken", xml), 2)
    assert info["ok"] == 0, info

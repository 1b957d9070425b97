"""CPU oracle: schedule simulator properties, numerics, golden vectors and the C baseline port."""
import ctypes
import glob
import os
import subprocess

import numpy as np
import pytest

from msccl_amd import xmlgen
from oracle import loader as L
from oracle import numerics as N
from oracle import plan as P
from oracle import sim as S
from tests.conftest import RCCL_XML_DIR, xml_ngpus
from tests.golden import make_golden as G

HERE = os.path.dirname(os.path.abspath(__file__))


def run(xml, n, coll, count, dt, op=0, inplace=True, mode="exact", seed=1):
    return G.run_case(xml, n, coll, count, dt, op, inplace, mode, seed)


# ------------------------------------------------------------------ exact-integer known answers
@pytest.mark.parametrize("xml,n,count,dt,inplace", [
    (lambda: xmlgen.allreduce_allpairs(2, 4, "LL"), 2, 4096 + 32, 7, True),
    (lambda: xmlgen.allreduce_allpairs(3, 2, "Simple"), 3, 18 * 100, 6, True),
    (lambda: xmlgen.allreduce_allpairs(8, 4, "LL", inplace=False), 8, 256 * 5, 9, False),
    (lambda: xmlgen.allreduce_ring(8, 4, "Simple"), 8, 32 * 257, 7, True),
    (lambda: xmlgen.allreduce_ring(5, 3, "LL", inplace=False), 5, 15 * 64, 8, False),
    (lambda: xmlgen.allreduce_oneshot(2, 1, "LL"), 2, 33, 7, True),
    (lambda: xmlgen.allreduce_oneshot(2, 4, "Simple"), 2, 4 * 1000, 7, True),
    (lambda: xmlgen.allreduce_oneshot(4, 2, "LL128"), 4, 2 * 300, 6, True),
    (lambda: xmlgen.allreduce_oneshot(8, 2, "LL", ordered=True), 8, 2 * 500, 7, True),
    (lambda: xmlgen.allreduce_oneshot(3, 1, "Simple", ordered=True), 3, 1000, 9, True),
])
def test_allreduce_exact_sum(xml, n, count, dt, inplace):
    ins, outs = run(xml(), n, L.ALLREDUCE, count, dt, inplace=inplace)
    want = sum(N.to_float64(dt, x) for x in ins)
    for r in range(n):
        assert np.array_equal(N.to_float64(dt, outs[r]), want)


def test_oneshot_two_ranks_bitwise_identical_across_ranks():
    """n = 2 one-shot: each rank folds fn(own, peer); commutative ops give both ranks the same bits."""
    ins, outs = run(xmlgen.allreduce_oneshot(2, 2, "LL"), 2, L.ALLREDUCE, 2 * 777, 7, mode="uniform")
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
    want = N.apply(0, 7, ins[0], ins[1])  # fp32 a + b, RNE
    assert np.array_equal(outs[0].view(np.uint32), np.asarray(want, np.float32).view(np.uint32))


@pytest.mark.parametrize("proto", ["LL", "LL128", "Simple"])
def test_oneshot_ordered_rank_order_fold(proto):
    """ordered one-shot: every rank holds the same bits, the left fold x0 (+) x1 (+) ... in rank
    order (LL / LL128: dst first; Simple: (s1 (+) ... ) (+) d, the same on every rank)."""
    n, dt = 5, 7
    ins, outs = run(xmlgen.allreduce_oneshot(n, 2, proto, ordered=True), n, L.ALLREDUCE, 2 * 999, dt,
                    mode="uniform")
    for r in range(1, n):
        assert np.array_equal(outs[0].view(np.uint32), outs[r].view(np.uint32))
    if proto != "Simple":
        want = ins[0]
        for q in range(1, n):
            want = N.apply(0, dt, want, ins[q])
        assert np.array_equal(outs[0].view(np.uint32), np.asarray(want, np.float32).view(np.uint32))


def test_reduce_scatter_allgather_exact():
    n, count = 8, 96
    ins, outs = run(xmlgen.reduce_scatter_allpairs(n, 2, "Simple"), n, L.REDUCE_SCATTER, count, 7, inplace=False)
    tot = sum(x.astype(np.float64) for x in ins)
    for r in range(n):
        assert np.array_equal(outs[r].astype(np.float64), tot[r * count:(r + 1) * count])
    ins, outs = run(xmlgen.allgather_allpairs(n, 2, "LL"), n, L.ALLGATHER, count, 7, inplace=False)
    for r in range(n):
        assert np.array_equal(outs[r], np.concatenate(ins))


def test_rccl_schedules_exact(rccl_xmls):
    for f in rccl_xmls:
        n = xml_ngpus(f)
        if n > 8:
            continue
        text = open(f).read()
        a = L.parse_xml(text, 0, n)
        ncpl = a.nchunksperloop
        if a.coll == L.ALLREDUCE:
            count = ncpl * 3
            if count * 2 >= a.maxBytes or count * 2 < a.minBytes:
                count = max(ncpl, (a.minBytes // 2 // ncpl + 1) * ncpl)
            ins, outs = run(text, n, L.ALLREDUCE, count, 6, inplace=bool(a.inplace))
            want = sum(N.to_float64(6, x) for x in ins)
            for r in range(n):
                assert np.array_equal(N.to_float64(6, outs[r]), want), f


def test_allpairs_ll_association_order():
    """Appendix B: LL all-pairs result for rank r's chunks is ((x_r + x_p0) + x_p1) ... with p ascending."""
    n, count = 4, 16 * 64
    ins, outs = run(xmlgen.allreduce_allpairs(n, 1, "LL"), n, L.ALLREDUCE, count, 7, mode="uniform")
    chunk = count // (n * n)
    idx = np.arange(count)
    owner = (idx // chunk // n) % n
    want = np.empty(count, np.float32)
    for r in range(n):
        acc = ins[r].copy()
        for p in range(n):
            if p != r:
                acc = acc + ins[p]
        want[owner == r] = acc[owner == r]
    for r in range(n):
        assert np.array_equal(outs[r], want)


def test_simple_big_chunk_dst_last_order():
    """Simple re with >= nthreads elements: ((s0 + s1) + ...) + d (prims_simple.h:258-263)."""
    n = 3
    count = n * n * 2048  # 2048 elements per chunk >= 544
    ins, outs = run(xmlgen.allreduce_allpairs(n, 1, "Simple"), n, L.ALLREDUCE, count, 7, mode="uniform")
    chunk = count // (n * n)
    owner = (np.arange(count) // chunk // n) % n
    want = np.empty(count, np.float32)
    for r in range(n):
        peers = [p for p in range(n) if p != r]
        acc = ins[peers[0]].copy()
        for p in peers[1:]:
            acc = acc + ins[p]
        acc = acc + ins[r]
        want[owner == r] = acc[owner == r]
    for r in range(n):
        assert np.array_equal(outs[r], want)


def test_deadlock_detected():
    bad = xmlgen.allreduce_allpairs(2, 1, "LL").replace('type="s" srcbuf="i" srcoff="2"', 'type="nop" srcbuf="i" srcoff="2"', 1)
    with pytest.raises((S.SimDeadlock, S.SimError, AssertionError, L.XmlError)):
        run(bad, 2, L.ALLREDUCE, 64, 7)


# ------------------------------------------------------------------ numerics
def test_fp16_sum_clamp_and_nan():
    x = np.array([60000, -60000, np.inf, np.nan, 1.0, 65504], np.float16)
    y = np.array([60000, -60000, 1.0, 1.0, 2.0, 16], np.float16)
    r = N.apply(N.SUM, 6, x, y)
    assert list(r.astype(np.float64)) == [65504.0, -65504.0, 65504.0, -65504.0, 3.0, 65504.0]


def test_bf16_rne():
    f = np.array([1.0 + 2 ** -8, 1.0 + 3 * 2 ** -8, -2.5], np.float32)
    b = N.f32_to_bf16(f)
    assert list(N.bf16_to_f32(b)) == [1.0, 1.0 + 2 ** -6, -2.5]


def test_ulp_distance():
    a = np.array([1.0, -1.0, 0.0], np.float32)
    b = np.nextafter(a, np.float32(np.inf))
    assert list(N.ulp_distance(7, a, b)) == [1, 1, 1]


@pytest.mark.parametrize("dt", [7, 6, 9])
def test_error_bound_vs_fp64_sum(dt):
    """Recursive-summation bound |s - exact| <= (n-1) u sum|x_i| against the fp64 sum."""
    n, count = 8, 256 * 8
    ins, outs = run(xmlgen.allreduce_allpairs(n, 4, "LL"), n, L.ALLREDUCE, count, dt, mode="uniform")
    xs = [N.to_float64(dt, x) for x in ins]
    exact = sum(xs)
    mag = sum(np.abs(x) for x in xs)
    u = {7: 2.0 ** -24, 6: 2.0 ** -11, 9: 2.0 ** -8}[dt]
    err = np.abs(N.to_float64(dt, outs[0]) - exact)
    assert np.all(err <= (n - 1) * u * mag * (1 + 1e-6) + 1e-30)


# ------------------------------------------------------------------ golden vectors
@pytest.mark.parametrize("case", G.CASES, ids=[c[0] for c in G.CASES])
def test_golden(case):
    name, xf, n, coll, count, dt, op, inplace, mode = case
    path = os.path.join(HERE, "golden", name + ".npz")
    try:
        xml = xf()
    except OSError:
        pytest.skip("source XML missing")
    z = np.load(path)
    ins, outs = G.run_case(xml, n, coll, count, dt, op, inplace, mode)
    assert np.array_equal(np.stack(ins), z["inputs"])
    assert np.array_equal(np.stack(outs).view(np.uint8), z["outputs"].view(np.uint8))


# ------------------------------------------------------------------ C port of the reduction
@pytest.fixture(scope="module")
def cpulib(tmp_path_factory):
    out = tmp_path_factory.mktemp("c") / "libcpu.so"
    src = os.path.join(os.path.dirname(HERE), "oracle", "cpu_allreduce.c")
    subprocess.check_call(["gcc", "-O2", "-fopenmp", "-shared", "-fPIC", src, "-o", str(out)])
    return ctypes.CDLL(str(out))


@pytest.mark.parametrize("dt,n", [(7, 2), (6, 8), (9, 4)])
def test_c_baseline_matches_simulator(cpulib, dt, n):
    count = n * n * 64
    ins, outs = run(xmlgen.allreduce_allpairs(n, 1, "LL"), n, L.ALLREDUCE, count, dt, mode="uniform")
    bufs = [x.copy() for x in ins]
    ptrs = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
    cpulib.cpu_allreduce_allpairs(ptrs, n, ctypes.c_long(count), ctypes.c_long(count // (n * n)), dt)
    for r in range(n):
        assert np.array_equal(bufs[r].view(np.uint8), outs[r].view(np.uint8))

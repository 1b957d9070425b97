"""The ring-fallback oracle (oracle/ring.py) against exact sums, and the product's ring plan
(plan.cc makeRingPlan via mscclAmdPlanJson) against the oracle's ring_params (CPU only)."""
import numpy as np
import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from oracle import loader as L
from oracle import ring as R

@pytest.fixture(autouse=True)
def _ring_algorithm(monkeypatch):
    """These cases pin the ring (small AllReduces take the tree by default: plan.cc makeRingPlan);
    the tree tests select it themselves."""
    monkeypatch.setenv("NCCL_ALGO", "Ring,Tree")
    monkeypatch.setenv("MSCCL_AMD_TREE_MAX_BYTES", "0")



@pytest.mark.parametrize("n", [2, 3, 5, 8])
@pytest.mark.parametrize("count", [1, 7, 1000, 70001, 300001])
def test_ring_oracle_exact(n, count):
    rng = np.random.default_rng(count + n)
    ins = [rng.integers(-4, 5, count).astype(np.float32) for _ in range(n)]
    want = np.sum(np.stack(ins).astype(np.float64), axis=0)
    outs, _ = R.run(L.ALLREDUCE, count, 7, 0, [x.copy() for x in ins], [None] * n, True)
    for o in outs:
        assert np.array_equal(o.astype(np.float64), want)
    big = [rng.integers(-4, 5, count * n).astype(np.float32) for _ in range(n)]
    tot = np.sum(np.stack(big), axis=0)
    outs, _ = R.run(L.REDUCE_SCATTER, count, 7, 0, [x.copy() for x in big], [None] * n, True)
    for r, o in enumerate(outs):
        assert np.array_equal(o, tot[r * count:(r + 1) * count])
    cat = np.concatenate([x[:count] for x in big])
    for ip in (True, False):
        outs, _ = R.run(L.ALLGATHER, count, 7, 0, [x[:count].copy() for x in big],
                        [np.zeros(count * n, np.float32) for _ in range(n)], ip)
        for o in outs:
            assert np.array_equal(o, cat)


def test_ring_oracle_association_order():
    """fp32 values whose sum depends on the order: the oracle follows the ring (chunk c starts at
    rank c+1, recv-reduce fn(peer, local) in LL), not a left fold."""
    n, count = 3, 3 * 1024
    ins = [np.full(count, v, np.float32) for v in (1e8, 1.0, -1e8)]
    outs, rp = R.run(L.ALLREDUCE, count, 7, 0, [x.copy() for x in ins], [None] * n, True)
    assert rp["proto"] == L.PROTO_LL
    vals = set(np.unique(outs[0]).tolist())
    assert vals <= {0.0, 1.0} and len(vals) == 2


CASES = [(L.ALLREDUCE, c, dt) for c in (1, 999, 1 << 16, 131073, 1 << 22, 50000001) for dt in (7, 6, 9, 0)] + \
        [(L.REDUCE_SCATTER, c, dt) for c in (1, 4097, 1 << 18, 3000001) for dt in (7, 9)] + \
        [(L.ALLGATHER, c, dt) for c in (1, 4097, 1 << 18, 3000001) for dt in (7, 6)]


@pytest.mark.parametrize("n", [2, 8])
@pytest.mark.parametrize("coll,count,dt", CASES)
def test_ring_plan_matches_oracle(tmp_path, n, coll, count, dt):
    p = tmp_path / "none.xml"
    p.write_text(xmlgen.allreduce_allpairs(n, 1, "LL", max_bytes=1))  # matches nothing
    prod = M.plan_json(str(p), 0, n, coll, count, dt, 0, coll != L.ALLGATHER)
    assert prod["algo"] == -1
    rp = R.ring_params(coll, count, dt, n)
    ring = prod["ring"]
    assert (ring["proto"], ring["channels"], ring["nthreads"], ring["size"], ring["dtype"], ring["nBytes"],
            ring["chunk"], ring["minChunk"], ring["lastChunk"]) == \
        (rp["proto"], rp["channels"], rp["nthreads"], rp["size"], rp["dtype"], rp["nbytes"], rp["chunk"],
         rp["min_chunk"], rp["last_chunk"])


def test_ring_plan_env(tmp_path, monkeypatch):
    p = tmp_path / "none.xml"
    p.write_text(xmlgen.allreduce_allpairs(2, 1, "LL", max_bytes=1))
    monkeypatch.setenv("MSCCL_AMD_RING_CHANNELS", "5")
    monkeypatch.setenv("NCCL_PROTO", "Simple")
    prod = M.plan_json(str(p), 0, 2, L.ALLREDUCE, 1000, 7, 0, True)["ring"]
    rp = R.ring_params(L.ALLREDUCE, 1000, 7, 2)
    assert prod["channels"] == rp["channels"] == 5
    assert prod["proto"] == rp["proto"] == L.PROTO_SIMPLE
    monkeypatch.setenv("MSCCL_AMD_RING_FALLBACK", "0")
    assert "ring" not in M.plan_json(str(p), 0, 2, L.ALLREDUCE, 1000, 7, 0, True)
    # PreMulSum (ncclAvg on floats) is never MSCCL-eligible but runs on the ring; SumPostDiv only
    # exists for integer types (reduce_kernel.h:498-520)
    monkeypatch.delenv("MSCCL_AMD_RING_FALLBACK")
    assert M.plan_json(str(p), 0, 2, L.ALLREDUCE, 1000, 7, 4, True)["algo"] == -1
    assert "ring" in M.plan_json(str(p), 0, 2, L.ALLREDUCE, 1000, 7, 4, True)
    assert "ring" in M.plan_json(str(p), 0, 2, L.ALLREDUCE, 1000, 2, 5, True)
    assert "ring" not in M.plan_json(str(p), 0, 2, L.ALLREDUCE, 1000, 7, 5, True)


from tests.golden import make_golden as G  # noqa: E402


@pytest.mark.parametrize("case", G.RING_CASES, ids=[c[0] for c in G.RING_CASES])
def test_ring_golden(case):
    import os
    name, n, coll, count, dt, op, inplace = case
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name + ".npz"))
    ins, outs = G.run_ring_case(n, coll, count, dt, op, inplace)
    assert np.array_equal(np.stack(ins), z["inputs"])
    assert np.array_equal(np.stack(outs).view(np.uint8), z["outputs"].view(np.uint8))


def test_avg_lowering_matches_reference_host_code():
    """hostToDevRedOp (enqueue.cc:1403-1431): integers -> SumPostDiv by n, floats -> PreMulSum by
    1/n rounded through float (half: __float2half(float(1.0/n)))."""
    from oracle import numerics as N
    assert N.avg_op(2, 3) == (N.SUMPOSTDIV, 3)
    assert N.avg_op(6, 3) == (N.PREMULSUM, 0x3555)          # 0.33325 in binary16
    assert N.avg_op(9, 3) == (N.PREMULSUM, 0x3EAB)          # bf16 RNE of float(1/3) 0x3eaaaaab
    assert N.avg_op(7, 8) == (N.PREMULSUM, 0x3E000000)      # 0.125f
    assert N.avg_op(8, 4) == (N.PREMULSUM, 0x3FD0000000000000)


def test_sumpostdiv_truncates_toward_zero():
    from oracle import numerics as N
    x = np.array([-7, 7, -1, 5, -128, 127], np.int8)
    assert N.post_op(N.SUMPOSTDIV, 0, x, 2).tolist() == [-3, 3, 0, 2, -64, 63]
    u = np.array([2 ** 64 - 1], np.uint64)
    assert int(N.post_op(N.SUMPOSTDIV, 5, u, 3)[0]) == (2 ** 64 - 1) // 3


@pytest.mark.parametrize("dt", [7, 6, 9, 2])
def test_ring_avg_is_the_mean_for_power_of_two_ranks(dt):
    """With 4 ranks and small-integer inputs every scaled value and partial sum is exact, so
    the ring's Avg must be exactly the mean (integers: the truncated mean)."""
    from oracle import numerics as N
    from oracle import ring as R
    from tests.gpu_harness import gen_inputs
    n, count = 4, 3001
    ins = gen_inputs(n, count, dt, 5, mode="exact")
    dev_op, arg = N.avg_op(dt, n)
    res, _ = R.run(L.ALLREDUCE, count, dt, dev_op, [x.copy() for x in ins], [None] * n, True, arg)
    tot = np.sum([N.to_float64(dt, x) for x in ins], axis=0)
    want = np.trunc(tot / n) if N.DTYPES[dt][2] == "int" else tot / n
    for r in range(n):
        assert np.array_equal(N.to_float64(dt, res[r]), want), r


@pytest.mark.parametrize("count,dt", [(1, 7), (999, 7), (40000, 6), (300001, 7), (5_000_000, 9)])
@pytest.mark.parametrize("n", [2, 3, 8])
def test_tree_plan_matches_product(tmp_path, monkeypatch, count, dt, n):
    """NCCL_ALGO=Tree: the product's tree plan (plan.cc makeTreePlan) equals the oracle's restatement
    of computeColl's tree chunk math and runTreeSplit's shrink."""
    p = tmp_path / "none.xml"
    p.write_text(xmlgen.allreduce_allpairs(2, 1, "LL", max_bytes=1))
    monkeypatch.setenv("NCCL_ALGO", "Tree")
    prod = M.plan_json(str(p), 0, n, L.ALLREDUCE, count, dt, 0, True)["ring"]
    rp = R.ring_params(L.ALLREDUCE, count, dt, n)
    assert rp["algo"] == "tree" and prod["coll"] == 4
    assert (prod["proto"], prod["channels"], prod["chunk"], prod["minChunk"], prod["nthreads"]) == \
        (rp["proto"], rp["channels"], rp["chunk"], rp["min_chunk"], rp["nthreads"])


@pytest.mark.parametrize("dt", [7, 6, 2])
@pytest.mark.parametrize("n", [2, 5])
def test_tree_oracle_exact_and_chain_order(monkeypatch, dt, n):
    """Exact-integer inputs give the exact sum on every rank; with LL the chain folds
    fn(peer, local) upward: ((x[n-1] + x[n-2]) + ...) + x[0]."""
    from tests.gpu_harness import gen_inputs
    from oracle import numerics as N
    monkeypatch.setenv("NCCL_ALGO", "Tree")
    count = 70001
    ins = gen_inputs(n, count, dt, 9, mode="exact")
    res, rp = R.run(L.ALLREDUCE, count, dt, 0, [x.copy() for x in ins], [None] * n, True)
    assert rp["algo"] == "tree"
    tot = np.sum([N.to_float64(dt, x) for x in ins], axis=0)
    for r in range(n):
        assert np.array_equal(N.to_float64(dt, res[r]), tot)
    ins = gen_inputs(n, 3001, 7, 4)
    res, rp = R.run(L.ALLREDUCE, 3001, 7, 0, [x.copy() for x in ins], [None] * n, True)
    acc = ins[n - 1]
    for r in range(n - 2, -1, -1):
        acc = N.apply(0, 7, acc, ins[r])
    assert np.array_equal(res[0].view(np.uint32), acc.view(np.uint32))


def test_flat_routing(tmp_path, monkeypatch):
    """Which fallback calls the one-hop fold kernel takes (plan.cc makeFlatTreePlan; "flat" is the
    collective it runs: 1 AllReduce, 2 ReduceScatter, 3 AllGather, 0 = the ring / chain tree)."""
    p = tmp_path / "none.xml"
    p.write_text(xmlgen.allreduce_allpairs(2, 1, "LL", max_bytes=1))
    monkeypatch.delenv("MSCCL_AMD_TREE_MAX_BYTES")

    def flat(n, coll, count, dt, op=0):
        return M.plan_json(str(p), 0, n, coll, count, dt, op, True)["ring"]["flat"]
    # ReduceScatter / AllGather: the LL range (512 KiB in all); pre / post ops keep the ring
    assert flat(8, L.REDUCE_SCATTER, 16384, 7) == 2
    assert flat(8, L.REDUCE_SCATTER, 16385, 7) == 0
    assert flat(8, L.REDUCE_SCATTER, 1000, 7, op=4) == 0
    assert flat(4, L.REDUCE_SCATTER, 1000, 2, op=3) == 2
    assert flat(16, L.ALLGATHER, 16384, 6) == 3
    assert flat(16, L.ALLGATHER, 16385, 6) == 0
    assert flat(17, L.ALLGATHER, 100, 6) == 0      # at most 16 ranks
    # AllReduce, Sum..Min: the tree takes the LL range where the flat tree runs it
    assert flat(8, L.ALLREDUCE, 131072, 7) == 1
    r = M.plan_json(str(p), 0, 8, L.ALLREDUCE, 131073, 7, 0, True)["ring"]
    assert r["flat"] == 0 and r["coll"] == 1
    assert flat(8, L.ALLREDUCE, 1000, 7, op=4) == 0
    # Avg (PreMulSum): the chain tree up to 16 KiB per rank, then the ring
    assert M.plan_json(str(p), 0, 8, L.ALLREDUCE, 32768, 7, 4, True)["ring"]["coll"] == 4
    assert M.plan_json(str(p), 0, 8, L.ALLREDUCE, 32769, 7, 4, True)["ring"]["coll"] == 1
    for cnt, op in ((131072, 0), (131073, 0), (32768, 4), (32769, 4)):
        want = "tree" if cnt in (131072, 32768) else "ring"
        assert R.ring_params(L.ALLREDUCE, cnt, 7, 8, op)["algo"] == want
    monkeypatch.setenv("MSCCL_AMD_TREE_MAX_BYTES", "1024")
    assert flat(2, L.REDUCE_SCATTER, 256, 7) == 2 and flat(2, L.REDUCE_SCATTER, 257, 7) == 0
    monkeypatch.setenv("MSCCL_AMD_TREE_FLAT", "0")
    assert flat(2, L.REDUCE_SCATTER, 256, 7) == 0 and flat(2, L.ALLREDUCE, 256, 7) == 0

"""Product selection + chunk math (plan.cc via mscclAmdPlanJson) == oracle plan (oracle/plan.py)."""
import os

import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from oracle import loader as L
from oracle import plan as P


@pytest.fixture(scope="module")
def xmls(tmp_path_factory):
    d = tmp_path_factory.mktemp("plan")
    out = {}
    specs = {
        "ap2ll": (xmlgen.allreduce_allpairs(2, 4, "LL", max_bytes=1 << 26), 2),
        "ap2s": (xmlgen.allreduce_allpairs(2, 8, "Simple", max_bytes=1 << 28), 2),
        "ap8ll": (xmlgen.allreduce_allpairs(8, 4, "LL", max_bytes=1 << 26), 8),
        "ring8": (xmlgen.allreduce_ring(8, 4, "Simple", max_bytes=(1 << 28) + 1), 8),
        "rs8": (xmlgen.reduce_scatter_allpairs(8, 2, "Simple"), 8),
        "ag8": (xmlgen.allgather_allpairs(8, 2, "LL"), 8),
    }
    for k, (x, n) in specs.items():
        p = d / (k + ".xml")
        p.write_text(x)
        out[k] = (str(p), n)
    return out


CASES = [
    ("ap2ll", L.ALLREDUCE, [32, 1024, 4096, 1 << 16, (1 << 20) + 16, 1 << 23], [7, 6, 9, 8, 0], True),
    ("ap2s", L.ALLREDUCE, [64, 4096, 1 << 20, 3 << 20, 1 << 25], [7, 6, 9], True),
    ("ap8ll", L.ALLREDUCE, [256, 1 << 14, 1 << 20, 1 << 24], [6, 7], True),
    ("ring8", L.ALLREDUCE, [32, 1 << 20, 1 << 27], [9, 7], True),
    ("rs8", L.REDUCE_SCATTER, [2, 1 << 10, 1 << 21], [7, 6], False),
    ("ag8", L.ALLGATHER, [2, 1 << 10, 1 << 20], [7, 2], False),
]


@pytest.mark.parametrize("key,coll,counts,dtypes,inplace", CASES)
def test_plan_matches_oracle(xmls, key, coll, counts, dtypes, inplace):
    path, n = xmls[key]
    algos = [L.load_xml(path, 0, n)]
    for count in counts:
        for dt in dtypes:
            for op in (0, 3):
                prod = M.plan_json(path, 0, n, coll, count, dt, op, inplace)
                call = P.Call(coll, count, dt, op, n, 0, inplace)
                idx = P.select(algos, call)
                if idx is None:
                    assert prod["algo"] == -1, (key, count, dt)
                    continue
                assert prod["algo"] == idx
                pl = P.make_plan(algos, call, idx)
                size_per = (pl.count * pl.size_multiplier) // pl.ncpl
                assert (prod["proto"], prod["nthreads"], prod["count"], prod["dtype"], prod["sizeMultiplier"],
                        prod["nBytes"], prod["maxAllowedCount"], prod["ncpl"], prod["sizePerChunk"]) == \
                    (pl.proto, pl.nthreads, pl.count, pl.dtype, pl.size_multiplier, pl.nbytes,
                     pl.max_allowed_count, pl.ncpl, size_per), (key, count, dt)
                iters = list(P.chunking(pl, [1, 1, 4, 4, 8, 8, 2, 4, 8, 2][pl.dtype]))
                assert prod["nIters"] == len(iters)


def test_selection_rules(xmls):
    path, n = xmls["ap2ll"]
    # not divisible by nchunksperloop (16) -> no match (reference: ring/tree fallback)
    assert M.plan_json(path, 0, n, L.ALLREDUCE, 24, 7, 0, True)["algo"] == -1
    # out of place against an in-place XML -> no match
    assert M.plan_json(path, 0, n, L.ALLREDUCE, 1024, 7, 0, False)["algo"] == -1
    # Avg is never MSCCL (tuning.cc:345)
    assert M.plan_json(path, 0, n, L.ALLREDUCE, 1024, 7, 4, True)["algo"] == -1
    # nBytes >= maxBytes -> no match
    assert M.plan_json(path, 0, n, L.ALLREDUCE, 1 << 24, 7, 0, True)["algo"] == -1
    # wrong collective
    assert M.plan_json(path, 0, n, L.REDUCE_SCATTER, 1024, 7, 0, True)["algo"] == -1


def test_first_matching_file_wins(xmls, tmp_path):
    small = tmp_path / "s.xml"
    small.write_text(xmlgen.allreduce_allpairs(2, 1, "LL", min_bytes=0, max_bytes=4096))
    big = tmp_path / "b.xml"
    big.write_text(xmlgen.allreduce_allpairs(2, 4, "Simple", min_bytes=4096, max_bytes=1 << 30))
    files = "%s:%s" % (small, big)
    assert M.plan_json(files, 0, 2, L.ALLREDUCE, 256, 7, 0, True)["algo"] == 0
    assert M.plan_json(files, 0, 2, L.ALLREDUCE, 1 << 16, 7, 0, True)["algo"] == 1


def test_env_buffsize_and_nthreads(xmls, monkeypatch):
    path, n = xmls["ap2ll"]
    monkeypatch.setenv("NCCL_NTHREADS", "256")
    monkeypatch.setenv("NCCL_LL_BUFFSIZE", str(1 << 18))
    prod = M.plan_json(path, 0, n, L.ALLREDUCE, 1 << 20, 7, 0, True)
    algos = [L.load_xml(path, 0, n)]
    call = P.Call(L.ALLREDUCE, 1 << 20, 7, 0, n, 0, True)
    pl = P.make_plan(algos, call, 0)
    assert prod["nthreads"] == pl.nthreads == 256
    assert prod["maxAllowedCount"] == pl.max_allowed_count
    assert prod["nIters"] == len(list(P.chunking(pl, 4)))

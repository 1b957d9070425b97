"""One-hop MSCCL AllReduce schedules lowered to the fold kernel on the GPU (msccl_amd/csrc/lower.cc).

A call of a schedule that lower.cc proves to be a one-hop fold (LL, op Sum..Min, at most
MSCCL_AMD_LOWER_MAX_BYTES per rank) runs mscclFoldKernel with the schedule's fold order.  Every
result here is compared bit for bit with oracle/sim.py running the XML itself (the reference's
interpreter semantics), and the comm info names the kernel that ran: last.small == 2 (the fold)
with last.algo the schedule's index, or 1 / 0 (the interpreter)."""
import os

import numpy as np
import pytest

from msccl_amd import xmlgen
from oracle import loader as L
from oracle import numerics as N
from tests.gpu_harness import CoResident, describe_mismatch, from_torch, gen_inputs, to_torch

pytestmark = pytest.mark.gpu
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "20")


def _bench():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    import bench
    return bench


def _case(cr, count, dt, seed, op=0, in_place=True):
    import torch
    dev = torch.device("cuda:0")
    ins = gen_inputs(cr.n, count, dt, seed)
    t = [to_torch(x, dev) for x in ins]
    outs = t if in_place else [torch.zeros_like(x) for x in t]
    torch.cuda.synchronize()
    cr.run(L.ALLREDUCE, count, dt, op, [x.data_ptr() for x in t], [x.data_ptr() for x in outs])
    gpu = [from_torch(x, N.storage(dt)) for x in outs]
    want, used = cr.oracle(L.ALLREDUCE, count, dt, op, ins, in_place)
    for r in range(cr.n):
        assert np.array_equal(gpu[r].view(np.uint8), want[r].view(np.uint8)), \
            "rank %d count %d dt %d op %d (schedule %s)\n%s" % (r, count, dt, op, used, describe_mismatch(gpu[r], want[r]))
    return cr.comms[0].info()["last"], used


@pytest.mark.parametrize("nbytes", [128, 1024, 4096, 16384, 32768])
def test_c2_pair_tiers_lowered(tmp_path, nbytes, monkeypatch):
    """C2 (2 ranks, fp32) through bench.py's tiers: calls up to the limit run the fold kernel
    (by default 4 KiB for 2 ranks; 16 KiB here), the rest the pair kernel on the flat connections
    (a lowered large call), or with MSCCL_AMD_LOWER_LARGE=0 the exchange-set small kernel."""
    monkeypatch.setenv("MSCCL_AMD_LOWER_MAX_BYTES", str(16 << 10))
    tiers = _bench().make_xmls(2, "LL", 16, str(tmp_path), _bench().PAIR_TIERS)
    for large in ("1", "0"):
        monkeypatch.setenv("MSCCL_AMD_LOWER_LARGE", large)
        with CoResident(2, [open(t[3]).read() for t in tiers], str(tmp_path)) as cr:
            for rep in range(3):
                last, used = _case(cr, nbytes // 4, 7, 10 * rep + nbytes % 89)
                if nbytes <= (16 << 10):
                    assert last["kernel"] == 2 and last["algo"] == used and last["ringColl"] == 5, last
                elif large == "1":
                    assert last["kernel"] == 3 and last["algo"] == used and last["ringColl"] == 5, last
                else:
                    assert last["small"] == 1 and last["set"] == 1 and last["algo"] == used, last


@pytest.mark.parametrize("nbytes", [128, 2048, 8192])
@pytest.mark.parametrize("dt", [6, 9])
def test_c3_oneshot_tier_lowered(tmp_path, nbytes, dt):
    """C3's small tier (8 ranks, rank-ordered one-shot x4, fp16 / bf16): the fold in rank order."""
    tiers = _bench().make_xmls(8, "LL", 4, str(tmp_path))
    with CoResident(8, [open(t[3]).read() for t in tiers], str(tmp_path)) as cr:
        last, used = _case(cr, nbytes // 2, dt, nbytes % 97)
        assert last["small"] == 2 and last["algo"] == used == 0, last


@pytest.mark.parametrize("op", [0, 1, 2, 3])
def test_unordered_oneshot_every_op(tmp_path, op, monkeypatch):
    """The unordered one-shot: every rank folds its own input first (a different order per rank,
    different fp16 bits per rank), out of place too (the pair exchange lowered by an explicit
    limit: by default it runs the pair kernel, init.cc: applySplits)."""
    monkeypatch.setenv("MSCCL_AMD_LOWER_MAX_BYTES", "4096")
    xml = xmlgen.allreduce_oneshot(4, 2, "LL")
    with CoResident(4, [xml], str(tmp_path)) as cr:
        last, _ = _case(cr, 2 * 1000, 6, 20 + op, op=op)
        assert last["small"] == 2, last
    xml = xmlgen.allreduce_pair_oneshot(2, "LL", inplace=False)
    with CoResident(2, [xml], str(tmp_path)) as cr:
        last, _ = _case(cr, 2 * 777, 9, 30 + op, op=op, in_place=False)
        assert last["small"] == 2, last


def test_knobs_and_limit(tmp_path, monkeypatch):
    """MSCCL_AMD_LOWER=0 keeps the interpreter; calls above MSCCL_AMD_LOWER_MAX_BYTES run the
    lowered pair (2 ranks), or with MSCCL_AMD_LOWER_LARGE=0 the interpreter too."""
    xml = xmlgen.allreduce_pair_oneshot(4, "LL")
    monkeypatch.setenv("MSCCL_AMD_LOWER", "0")
    with CoResident(2, [xml], str(tmp_path)) as cr:
        last, _ = _case(cr, 1024, 7, 1)
        assert last["small"] == 1, last
    monkeypatch.setenv("MSCCL_AMD_LOWER", "1")
    monkeypatch.setenv("MSCCL_AMD_LOWER_MAX_BYTES", "4096")
    with CoResident(2, [xml], str(tmp_path)) as cr:
        assert _case(cr, 1024, 7, 2)[0]["kernel"] == 2
        assert _case(cr, 1028, 7, 3)[0]["kernel"] == 3
    monkeypatch.setenv("MSCCL_AMD_LOWER_LARGE", "0")
    with CoResident(2, [xml], str(tmp_path)) as cr:
        assert _case(cr, 1024, 7, 2)[0]["kernel"] == 2
        # not lowered: the schedule's own connections, the pair kernel (pair form, one pass)
        last = _case(cr, 1028, 7, 3)[0]
        assert last["kernel"] == 3 and last["ringColl"] == 0, last


def test_lowered_interpreted_and_flat_calls_interleave(tmp_path, monkeypatch):
    """The lowered schedule shares the flat connections with the fallback's flat tree, and its
    own connections stay with its interpreted calls: 200 launches mixing the three, across the
    8-bit LL flag wrap and cleanup (MSCCL_AMD_TEST_LL_CLEANUP=1), every result bit-exact."""
    monkeypatch.setenv("MSCCL_AMD_TEST_LL_CLEANUP", "1")
    xml = xmlgen.allreduce_oneshot(4, 2, "LL", ordered=True, max_bytes=1 << 20)
    with CoResident(4, [xml], str(tmp_path)) as cr:
        kinds = set()
        for it in range(200):
            k = it % 3
            count = (2048, 2 * 40000, 2 * 3001 + 1)[k]   # lowered, interpreted, no schedule (flat tree)
            last, used = _case(cr, count, 6, it)
            kinds.add((k, last["small"] == 2, used))   # the interpreted call: general kernel (3 iterations)
        assert kinds == {(0, True, 0), (1, False, 0), (2, True, "ring")}, kinds


RCCL = "/opt/rocm/share/rccl/msccl-algorithms"


@pytest.mark.parametrize("nbytes", [512, 4096, 8192, 32768])
def test_rccl_allpairs_lowered_with_chunk_classes(tmp_path, nbytes):
    """RCCL's shipped msccl-tools all-pairs (8n LL 32 tb, fp16): its 256 chunks fold in 7 orders
    (each chunk's owner first), the fold kernel picks each pack's order by its chunk.  512 B is
    one element per chunk, not whole 16-B packs: that call keeps the interpreter."""
    p = os.path.join(RCCL, "allreduce-allpairs-8n-ll-32tb.xml")
    if not os.path.exists(p):
        pytest.skip("fixture missing")
    with CoResident(8, [open(p).read()], str(tmp_path)) as cr:
        for rep in range(2):
            last, used = _case(cr, nbytes // 2, 6, rep + nbytes % 83)
            assert (last["small"] == 2) == (nbytes >= 4096) and last["algo"] == used == 0, last


@pytest.mark.parametrize("n,count,dt,lowered", [(8, 2 * 64 * 8 * 8, 6, True), (4, 16 * 40, 7, True),
                                                 (4, 16 * 41, 7, False),
                                                 (8, 64 * 1024, 6, True)])   # 128 KiB: 16 fold workgroups
def test_allpairs_classes_and_whole_packs(tmp_path, n, count, dt, lowered):
    """The two-phase all-pairs: lowered when every chunk is whole 16-B packs (a pack folds in one
    chunk's order); 41 floats per chunk are not, and the call keeps the interpreter."""
    xml = xmlgen.allreduce_allpairs(n, 1, "LL", inplace=False)
    with CoResident(n, [xml], str(tmp_path)) as cr:
        last, _ = _case(cr, count, dt, count % 71, in_place=False)
        assert (last["small"] == 2) == lowered, last


@pytest.mark.parametrize("inst", [1, 2])
def test_ring_lowered_per_start_class(tmp_path, inst):
    """An 8-rank LL ring of 1 or 2 rings: each chunk folds along its ring from the rank after its
    owner (8 / 16 classes); the fold kernel gives the ring's bits at small sizes."""
    xml = xmlgen.allreduce_ring(8, inst, "LL")
    with CoResident(8, [xml], str(tmp_path)) as cr:
        for count, dt in ((8 * inst * 64, 6), (8 * inst * 8 * 37, 9)):
            last, _ = _case(cr, count, dt, count % 53)
            assert last["small"] == 2, last


@pytest.mark.parametrize("dt", [6, 7])
def test_lowered_fold_nan_positions(tmp_path, monkeypatch, dt):
    """NaN payloads are outside the fold's bit-exact claim (with two NaN operands
    IEEE add returns one payload by operand order).  What holds: the lowered call gives a NaN
    exactly where the interpreted schedule does, and every other element bit for bit."""
    import torch
    n, count = 8, 4096
    xml = xmlgen.allreduce_allpairs(n, 1, "LL")
    ins = gen_inputs(n, count, dt, 77)
    bits = {6: np.uint16, 7: np.uint32}[dt]
    quiet = {6: 0x7E00, 7: 0x7FC00000}[dt]
    for r in range(n):
        v = ins[r].view(bits)
        v[r::97] = quiet | (r + 1)            # a NaN payload per rank, at positions that overlap
        v[(3 * r) % 11::131] = quiet | 0x100 | r
    results = {}
    for lower in ("1", "0"):
        monkeypatch.setenv("MSCCL_AMD_LOWER", lower)
        with CoResident(n, [xml], str(tmp_path)) as cr:
            t = [to_torch(x, torch.device("cuda:0")) for x in ins]
            torch.cuda.synchronize()
            cr.run(L.ALLREDUCE, count, dt, 0, [x.data_ptr() for x in t], [x.data_ptr() for x in t])
            results[lower] = [from_torch(x, N.storage(dt)) for x in t]
            assert cr.comms[0].info()["last"]["small"] == (2 if lower == "1" else 1)
    for r in range(n):
        a, b = results["1"][r], results["0"][r]
        fa = a.view(np.float16 if dt == 6 else np.float32)
        fb = b.view(np.float16 if dt == 6 else np.float32)
        assert np.array_equal(np.isnan(fa), np.isnan(fb)), "rank %d NaN positions differ" % r
        keep = ~np.isnan(fa)
        assert np.array_equal(a.view(bits)[keep], b.view(bits)[keep]), "rank %d non-NaN bits differ" % r
        # fp32 keeps NaN; the fp16 sum clamps it to -65504 (numerics: the reference's __hadd with
        # the clamp), so there the check is that both forms clamp the same elements
        assert np.isnan(fa).sum() > 0 if dt == 7 else (fa == -65504).sum() > 0

"""Lowered large calls (plan.cc: lowerToFoldPlan, MSCCL_AMD_LOWER_LARGE): the msccl-tools two-phase
all-pairs without its scratch round trip.

Above the fold's limit a lowered schedule (lower.cc) runs
  * with 2 ranks as the pair exchange on the flat connections (mscclPairKernel, kernel 3): every
    rank sends its input and folds the peer's copy into its own, one hop;
  * with more ranks, when every rank's result chunk is the same fold and the ranks own equal shares
    (lower.h: FoldLowering::twoPhase), as the two-phase fold (mscclTwoPhaseKernel, kernel 4): each
    owner folds its chunks straight from the peers' FIFO lines in the schedule's `re` order and
    sends the result on.
Every result is compared bit for bit with oracle/sim.py running the XML as written (the
reference's interpreter semantics: scratch, `re` order, the copies back), and the comm info names
the kernel that ran (last.kernel)."""
import os

import numpy as np
import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from oracle import loader as L
from oracle import numerics as N
from tests.gpu_harness import CoResident, describe_mismatch, from_torch, gen_inputs, to_torch

pytestmark = pytest.mark.gpu
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "20")

RCCL_32TB = "/opt/rocm/share/rccl/msccl-algorithms/allreduce-allpairs-8n-ll-32tb.xml"


def _case(cr, count, dt, seed, op=0, in_place=True, mode="uniform"):
    import torch
    dev = torch.device("cuda:0")
    ins = gen_inputs(cr.n, count, dt, seed, mode)
    t = [to_torch(x, dev) for x in ins]
    outs = t if in_place else [torch.full_like(x, 7) for x in t]
    torch.cuda.synchronize()
    cr.run(L.ALLREDUCE, count, dt, op, [x.data_ptr() for x in t], [x.data_ptr() for x in outs])
    gpu = [from_torch(x, N.storage(dt)) for x in outs]
    want, used = cr.oracle(L.ALLREDUCE, count, dt, op, ins, in_place)
    for r in range(cr.n):
        assert np.array_equal(gpu[r].view(np.uint8), want[r].view(np.uint8)), \
            "rank %d count %d dt %d op %d (schedule %s)\n%s" % (r, count, dt, op, used,
                                                               describe_mismatch(gpu[r], want[r]))
    return [c.info()["last"] for c in cr.comms], used


@pytest.mark.parametrize("nbytes", [8 << 10, 64 << 10, 1 << 20, 4 << 20, 32 << 20])
@pytest.mark.parametrize("in_place", [True, False])
def test_two_rank_allpairs_runs_the_pair_exchange(tmp_path, nbytes, in_place):
    """The msccl-tools two-phase all-pairs of 2 ranks (x16, the bench's secondary line): above 4 KiB
    the pair kernel on the flat connections, the XML's values."""
    xml = xmlgen.allreduce_allpairs(2, 16, "LL", inplace=in_place)
    with CoResident(2, [xml], str(tmp_path)) as cr:
        for rep in range(2):
            last, used = _case(cr, nbytes // 4, 7, rep + nbytes % 89, in_place=in_place)
            assert all(l["kernel"] == 3 and l["ringColl"] == 5 and l["algo"] == 0 for l in last), last


@pytest.mark.parametrize("nbytes", [256 << 10, 1 << 20, 4 << 20, 32 << 20])
@pytest.mark.parametrize("inst", [1, 4, 8])
def test_eight_rank_allpairs_runs_two_phase(tmp_path, nbytes, inst):
    """C3's two-phase all-pairs (8 ranks, fp16; x4 and x8 are the bench's tiers): the two-phase fold."""
    xml = xmlgen.allreduce_allpairs(8, inst, "LL")
    with CoResident(8, [xml], str(tmp_path)) as cr:
        last, used = _case(cr, nbytes // 2, 6, inst + nbytes % 83)
        assert all(l["kernel"] == 4 and l["algo"] == 0 for l in last), last


@pytest.mark.parametrize("nbytes", [256 << 10, 2 << 20, 32 << 20])
def test_rccl_allpairs_32tb_runs_two_phase(tmp_path, nbytes):
    """RCCL's shipped allreduce-allpairs-8n-ll-32tb (its maxBytes raised as the bench does): 256
    chunks, 8 owners, 8 fold orders; the two-phase fold gives the file's values."""
    if not os.path.exists(RCCL_32TB):
        pytest.skip("fixture missing")
    xml = open(RCCL_32TB).read().replace('maxBytes="65536"', 'maxBytes="%d"' % ((32 << 20) + 1))
    with CoResident(8, [xml], str(tmp_path)) as cr:
        last, used = _case(cr, nbytes // 2, 6, nbytes % 79)
        assert all(l["kernel"] == 4 for l in last), last


@pytest.mark.parametrize("n,inst,count,dt,op", [
    (4, 2, 32 * 8192, 7, 0), (4, 2, 32 * 8192, 7, 1), (4, 2, 32 * 8192, 7, 2), (4, 2, 32 * 8192, 7, 3),
    (3, 4, 36 * 4096, 9, 0), (8, 2, 128 * 2048, 2, 0), (16, 1, 256 * 1024, 6, 3), (5, 1, 25 * 8000, 8, 0),
    (8, 1, 64 * 1031 * 16, 0, 0), (6, 2, 72 * 2048, 3, 2)])
def test_two_phase_types_ops_and_rank_counts(tmp_path, n, inst, count, dt, op):
    """Every op, integer and float types, rank counts that are not powers of two (3, 5, 6) and 16,
    chunk sizes that are not powers of two (the magic division by the packs per chunk)."""
    xml = xmlgen.allreduce_allpairs(n, inst, "LL")
    with CoResident(n, [xml], str(tmp_path)) as cr:
        last, _ = _case(cr, count, dt, count % 97 + op, op=op)
        assert all(l["kernel"] == 4 for l in last), last


def test_two_phase_out_of_place(tmp_path):
    xml = xmlgen.allreduce_allpairs(8, 2, "LL", inplace=False)
    with CoResident(8, [xml], str(tmp_path)) as cr:
        last, _ = _case(cr, 128 * 4096, 6, 5, in_place=False)
        assert all(l["kernel"] == 4 for l in last), last


def test_not_whole_packs_keeps_the_interpreter(tmp_path):
    """10497 floats per chunk are not whole 16-B packs: the interpreter (its scratch form)."""
    xml = xmlgen.allreduce_allpairs(4, 1, "LL")
    with CoResident(4, [xml], str(tmp_path)) as cr:
        last, _ = _case(cr, 16 * 10497, 7, 3)
        assert all(l["kernel"] in (0, 1) for l in last), last


def test_knob_keeps_the_interpreter(tmp_path, monkeypatch):
    monkeypatch.setenv("MSCCL_AMD_LOWER_LARGE", "0")
    with CoResident(8, [xmlgen.allreduce_allpairs(8, 1, "LL")], str(tmp_path)) as cr:
        last, _ = _case(cr, 1 << 19, 6, 3)
        assert all(l["kernel"] in (0, 1) for l in last), last
    with CoResident(2, [xmlgen.allreduce_allpairs(2, 16, "LL")], str(tmp_path)) as cr:
        last, _ = _case(cr, 1 << 18, 7, 4)
        assert all(l["kernel"] in (0, 1) for l in last), last


def test_lowered_kernels_interleave_across_flag_wrap(tmp_path, monkeypatch):
    """One communicator set mixing, launch after launch, the fold (small calls), the two-phase fold
    (large calls), the interpreter (a call that is not whole packs) and the fallback's flat tree
    (no schedule matches): 120 launches across the 8-bit LL flag wrap and cleanup
    (MSCCL_AMD_TEST_LL_CLEANUP=1) on the shared flat connections, every result bit-exact."""
    monkeypatch.setenv("MSCCL_AMD_TEST_LL_CLEANUP", "1")
    xml = xmlgen.allreduce_allpairs(4, 2, "LL", max_bytes=1 << 24)
    with CoResident(4, [xml], str(tmp_path)) as cr:
        kinds = set()
        for it in range(120):
            k = it % 4
            count = (32 * 64, 32 * 8192 + 32 * 64 * (it % 3), 32 * 1001 * 8 + 32 * 3, 2 * 3001 + 1)[k]
            last, used = _case(cr, count, 7, it, mode="exact" if k == 1 else "uniform")
            kinds.add((k, 1 if k == 2 and last[0]["kernel"] in (0, 1) else last[0]["kernel"]))  # 2: general or small
        assert kinds == {(0, 2), (1, 4), (2, 1), (3, 2)}, kinds


def test_two_rank_pair_lowering_interleaves_with_interpreter_and_fold(tmp_path, monkeypatch):
    """2 ranks: the lowered pair (large), the fold (up to 4 KiB) and the interpreter (the pair
    exchange's own thread blocks, a call of whole packs but a partial last iteration: 1 MiB + 4 B
    is not divisible by 64 chunks -> ring fallback) in one sequence, across the flag wrap."""
    monkeypatch.setenv("MSCCL_AMD_TEST_LL_CLEANUP", "1")
    xml = xmlgen.allreduce_allpairs(2, 16, "LL")
    with CoResident(2, [xml], str(tmp_path)) as cr:
        kinds = set()
        for it in range(90):
            k = it % 3
            count = (256, (1 << 18) + 64 * (it % 5), (1 << 18) + 1)[k]
            last, used = _case(cr, count, 7, it)
            kinds.add((k, last[0]["kernel"]))
        assert (0, 2) in kinds and (1, 3) in kinds, kinds


def _mp_proc(rank, world, xml_path, count, dt, q_in, q_out):
    import torch
    os.environ["MSCCL_XML_FILES"] = xml_path
    os.environ["MSCCL_AMD_TIMEOUT_SEC"] = "30"
    torch.cuda.set_device(0)
    uid = M.get_unique_id() if rank == 0 else None
    if rank == 0:
        for _ in range(world - 1):
            q_in.put(uid)
    else:
        uid = q_in.get(timeout=60)
    x = gen_inputs(world, count, dt, 9, "exact")[rank]
    comm = M.Comm.init_rank(world, uid, rank)
    t = to_torch(x, torch.device("cuda:0"))
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        comm.all_reduce(t.data_ptr(), t.data_ptr(), count, dt, M.SUM, s)
    torch.cuda.synchronize()
    err = comm.async_error()
    last = comm.info()["last"]
    out = t.cpu().numpy()
    comm.destroy()
    q_out.put((rank, err, last["kernel"], out))


@pytest.mark.parametrize("world,inst,count,want", [(2, 16, 1 << 20, 3), (4, 2, 1 << 19, 4)])
def test_lowered_large_across_processes(tmp_path, world, inst, count, want):
    """One process per rank (hipIpc flat connections): the lowered pair and the two-phase fold,
    three calls in a row, exact integers (every order gives the same sum)."""
    import torch.multiprocessing as mp
    xml = xmlgen.allreduce_allpairs(world, inst, "LL")
    p = tmp_path / "ap.xml"
    p.write_text(xml)
    ctx = mp.get_context("spawn")
    q_in, q_out = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=_mp_proc, args=(r, world, str(p), count, 7, q_in, q_out)) for r in range(world)]
    for pr in ps:
        pr.start()
    res = {}
    for _ in range(world):
        r, err, kernel, out = q_out.get(timeout=300)
        res[r] = (err, kernel, out)
    for pr in ps:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    ins = gen_inputs(world, count, 7, 9, "exact")
    want_v = np.sum([x.astype(np.float64) for x in ins], axis=0) * world ** 2
    for r in range(world):
        assert res[r][0] == 0 and res[r][1] == want, (r, res[r][:2])
        assert np.array_equal(res[r][2].astype(np.float64), want_v), r

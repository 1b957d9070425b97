"""The small-call kernel (interpreter.h: runSmall, enqueue.cc: smallEligible).

A launch whose calls are one LL interpreter iteration of an MSCCL schedule runs
mscclSmallKernel.  It must give the reference's bits (oracle) exactly like the general kernel,
the two must agree bit for bit, and two ranks that run different kernels must still
interoperate (they cut every transfer into the same FIFO steps)."""
import os

import numpy as np
import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from oracle import loader as L
from tests.gpu_harness import CoResident, describe_mismatch, gen_inputs, to_torch, from_torch
from oracle import numerics as N

pytestmark = pytest.mark.gpu
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "20")


@pytest.fixture(autouse=True)
def _interpreter_kernels(monkeypatch):
    """These tests pin the interpreter's kernels: lowered schedules' large calls (the pair kernel on
    the flat connections, the two-phase fold: tests/test_gpu_twophase.py) stay off."""
    monkeypatch.setenv("MSCCL_AMD_LOWER_LARGE", "0")

SCHEDULES = {
    "pair2": (2, lambda: xmlgen.allreduce_pair_oneshot(1, "LL")),
    "allpairs8": (8, lambda: xmlgen.allreduce_allpairs(8, 1, "LL")),   # C3's form: reductions + deps
    "ring4": (4, lambda: xmlgen.allreduce_ring(4, 1, "LL")),
}


def _run(cr, count, dt, op, seed):
    import torch
    dev = torch.device("cuda:0")
    ins = gen_inputs(cr.n, count, dt, seed)
    t = [to_torch(x, dev) for x in ins]
    torch.cuda.synchronize()
    p = [x.data_ptr() for x in t]
    cr.run(L.ALLREDUCE, count, dt, op, p, p)
    return ins, [from_torch(x, N.storage(dt)) for x in t], [c.info()["last"] for c in cr.comms]


@pytest.mark.parametrize("name", sorted(SCHEDULES))
@pytest.mark.parametrize("count,dt,op", [(64, 7, 0), (320, 7, 2), (192, 7, 0), (1024, 6, 0), (16384, 9, 0),
                                         (8192, 7, 3)])
def test_small_kernel_matches_oracle_and_general(name, count, dt, op, tmp_path, monkeypatch):
    monkeypatch.setenv("MSCCL_AMD_LOWER", "0")   # the interpreter kernels, not the one-hop fold
    n, gen = SCHEDULES[name]
    xml = gen()
    xp = tmp_path / "s.xml"
    xp.write_text(xml)
    one_iter = M.plan_json(str(xp), 0, n, L.ALLREDUCE, count, dt, op, True)["nIters"] == 1
    outs = {}
    for small in ("1", "0"):
        monkeypatch.setenv("MSCCL_AMD_SMALL_KERNEL", small)
        with CoResident(n, [xml], str(tmp_path)) as cr:
            ins, got, last = _run(cr, count, dt, op, seed=11)
            if small == "0":
                assert all(l["small"] == 0 for l in last), last
            elif one_iter:  # several iterations may still run as one merged pass (small too)
                assert all(l["small"] == 1 for l in last), last
            want, idx = cr.oracle(L.ALLREDUCE, count, dt, op, ins, True)
            assert idx == 0
            for r in range(n):
                assert np.array_equal(got[r].view(np.uint8), want[r].view(np.uint8)), \
                    "small=%s rank %d: %s" % (small, r, describe_mismatch(got[r], want[r]))
            outs[small] = got
    for r in range(n):
        assert np.array_equal(outs["1"][r].view(np.uint8), outs["0"][r].view(np.uint8))


def test_partial_last_iteration_takes_general_kernel(tmp_path, monkeypatch):
    """A partial last iteration (passes of unequal size): the general kernel runs (and still
    matches the oracle)."""
    monkeypatch.setenv("MSCCL_AMD_SMALL_KERNEL", "1")
    xml = xmlgen.allreduce_pair_oneshot(1, "LL")
    with CoResident(2, [xml], str(tmp_path)) as cr:
        count = (1 << 20) + 64
        ins, got, last = _run(cr, count, 7, 0, seed=3)
        assert all(l["small"] == 0 for l in last), last
        want, _ = cr.oracle(L.ALLREDUCE, count, 7, 0, ins, True)
        for r in range(2):
            assert np.array_equal(got[r].view(np.uint32), want[r].view(np.uint32))


@pytest.mark.parametrize("count", [1 << 16, 1 << 17, 1 << 19])
def test_merged_pass_takes_small_kernel(tmp_path, monkeypatch, count):
    """Full iterations merged into equal passes (8, 16 and 64 LL iterations of the 16-instance
    pair schedule, the bench's 4, 8 and 32 MiB points; 64 runs as two passes of 32): the small
    kernel, bit-equal to the oracle."""
    monkeypatch.setenv("MSCCL_AMD_SMALL_KERNEL", "1")
    xml = xmlgen.allreduce_pair_oneshot(16, "LL")
    xp = tmp_path / "p.xml"
    xp.write_text(xml)
    assert M.plan_json(str(xp), 0, 2, L.ALLREDUCE, count * 16, 7, 0, True)["nIters"] > 1
    with CoResident(2, [xml], str(tmp_path)) as cr:
        ins, got, last = _run(cr, count * 16, 7, 0, seed=5)
        assert all(l["small"] == 1 for l in last), last
        want, _ = cr.oracle(L.ALLREDUCE, count * 16, 7, 0, ins, True)
        for r in range(2):
            assert np.array_equal(got[r].view(np.uint32), want[r].view(np.uint32))


def _mixed_proc(rank, world, xml_path, count, small, q_in, q_out):
    import torch
    os.environ["MSCCL_XML_FILES"] = xml_path
    os.environ["MSCCL_AMD_TIMEOUT_SEC"] = "30"
    os.environ["MSCCL_AMD_SMALL_KERNEL"] = small
    torch.cuda.set_device(0)
    uid = M.get_unique_id() if rank == 0 else None
    if rank == 0:
        for _ in range(world - 1):
            q_in.put(uid)
    else:
        uid = q_in.get(timeout=60)
    x = gen_inputs(world, count, 7, 9)[rank]
    comm = M.Comm.init_rank(world, uid, rank)
    t = to_torch(x, torch.device("cuda:0"))
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(5):
        comm.all_reduce(t.data_ptr(), t.data_ptr(), count, M.FLOAT32, M.SUM, s)
    torch.cuda.synchronize()
    err = comm.async_error()
    last = comm.info()["last"]
    out = t.cpu().numpy()
    comm.destroy()
    q_out.put((rank, err, last["small"], out))


def test_mixed_kernels_across_processes(tmp_path):
    """Rank 0 runs the small kernel, rank 1 the general one (MSCCL_AMD_SMALL_KERNEL is a
    rank-local choice): the FIFO steps still line up and the values are the reference's."""
    import torch.multiprocessing as mp
    from oracle import plan as P, sim as S
    world, count = 2, 3000  # 375 elements per chunk: not whole 16-B packs
    xml = xmlgen.allreduce_allpairs(world, 2, "LL")
    p = tmp_path / "ap.xml"
    p.write_text(xml)
    ctx = mp.get_context("spawn")
    q_in, q_out = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=_mixed_proc, args=(r, world, str(p), count, "1" if r == 0 else "0", q_in, q_out))
          for r in range(world)]
    for pr in ps:
        pr.start()
    res = {}
    for _ in range(world):
        r, err, small, out = q_out.get(timeout=300)
        res[r] = (err, small, out)
    for pr in ps:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert res[0][1] == 1 and res[1][1] == 0
    algos = [L.parse_xml(xml, r, world) for r in range(world)]
    call = P.Call(L.ALLREDUCE, count, 7, 0, world, 0, True)
    plan = P.make_plan([algos[0]], call, 0)
    ins = gen_inputs(world, count, 7, 9)
    for _ in range(5):
        ins, _st = S.run(algos, plan, ins, [None] * world, L.ALLREDUCE, True)
    for r in range(world):
        assert res[r][0] == 0
        assert np.array_equal(res[r][2].view(np.uint32), np.asarray(ins[r]).view(np.uint32))


@pytest.mark.parametrize("count,split", [(1 << 20, 4), (1 << 21, 8), (1 << 23, 8)])
def test_two_rank_wide_split_by_call_size(tmp_path, count, split):
    """Two co-resident ranks' LL schedules get the wide workgroup budget (plan.h: kWideSplitMinBytes):
    the 2-rank two-phase all-pairs x16 (32 thread blocks) runs split 8 while every workgroup moves
    32 KiB or more (8 and 32 MiB), split 4 below (4 MiB); the oracle's values either way."""
    xml = xmlgen.allreduce_allpairs(2, 16, "LL")
    with CoResident(2, [xml], str(tmp_path)) as cr:
        ins, got, last = _run(cr, count, 7, 0, seed=count % 97)
        assert all(l["split"] == split for l in last), last
        want, _ = cr.oracle(L.ALLREDUCE, count, 7, 0, ins, True)
        for r in range(2):
            assert np.array_equal(got[r].view(np.uint32), want[r].view(np.uint32))


def _uneven_pair_xml(inst: int) -> str:
    """The 2-rank pair exchange (s, rrc per thread block) where rank 0 also runs `inst` thread
    blocks of local copies (input chunk k to its scratch: value-neutral): the ranks run different
    numbers of thread blocks (the reference computes nBlocks per gpu, topo.cc:1173-1185)."""
    from msccl_amd.xmlgen import _Tb, _emit
    gpus = {}
    for r in range(2):
        tbs = []
        for k in range(inst):
            tb = _Tb(k, 1 - r, 1 - r, k)
            tb.add("s", "i", k, "i", k, 1)
            tb.add("rrc", "i", k, "i", k, 1)
            tbs.append(tb)
        if r == 0:
            for k in range(inst):
                tb = _Tb(inst + k, -1, -1, k)
                tb.add("cpy", "i", k, "s", k, 1)
                tbs.append(tb)
        gpus[r] = (inst, 0, inst if r == 0 else 0, tbs)
    return _emit("uneven_pair", "LL", inst, inst, 2, "allreduce", True, gpus, 0, 1 << 40)


@pytest.mark.parametrize("nbytes", [6 << 20, 3 << 20, 12 << 20])
def test_wide_split_agrees_when_ranks_run_different_thread_block_counts(tmp_path, nbytes):
    """the wide-split step-back compared against the rank's own thread-block
    count.  Rank 0 runs 32 thread blocks, rank 1 16: at 6 MiB rank 0's count stepped its split back
    to 4 while rank 1 kept 8, and the two ends of every sub-connection owned different packs (a hang
    or wrong data).  Both now use the most over every rank's program (algoMaxBlocks); the oracle's
    values at sizes inside and around the window."""
    xml = _uneven_pair_xml(16)
    with CoResident(2, [xml], str(tmp_path)) as cr:
        ins, got, last = _run(cr, nbytes // 4, 7, 0, seed=nbytes % 89)
        assert last[0]["split"] == last[1]["split"], last
        want, _ = cr.oracle(L.ALLREDUCE, nbytes // 4, 7, 0, ins, True)
        for r in range(2):
            assert np.array_equal(got[r].view(np.uint32), want[r].view(np.uint32)), \
                "rank %d: %s" % (r, describe_mismatch(got[r], want[r]))

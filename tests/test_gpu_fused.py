"""Fused s + rrc exchanges (transport.cc: fusableTbs, interpreter.h: llFusedOp).

A thread block whose first FIFO transfers are `s` then `rrc` of the same source chunks with one
peer runs both as one pass over its source when the peer's thread block on that connection has
the same shape (agreed at init).  The values must stay those of s then rrc (the oracle's), for
every size, type, op, in and out of place; both ends must agree before fusing (an asymmetric
exchange would deadlock fused); and a fused rank must interoperate with an unfused one."""
import os

import numpy as np
import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from msccl_amd.xmlgen import _Tb, _emit
from oracle import loader as L
from tests.gpu_harness import CoResident, describe_mismatch, gen_inputs, run_collective, to_torch

pytestmark = pytest.mark.gpu
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "20")


@pytest.fixture(autouse=True)
def _interpreter_kernels(monkeypatch):
    """These tests pin the interpreter's fused exchange and the pair kernel on the schedules' own
    connections: lowered large calls (tests/test_gpu_twophase.py) stay off."""
    monkeypatch.setenv("MSCCL_AMD_LOWER_LARGE", "0")


def _check(got, want, what):
    for r in range(len(want)):
        assert np.array_equal(np.asarray(got[r]).view(np.uint8), np.asarray(want[r]).view(np.uint8)), \
            "%s rank %d: %s" % (what, r, describe_mismatch(got[r], want[r]))


def test_pair_exchange_is_fused_and_allpairs_is_not(tmp_path, monkeypatch):
    monkeypatch.delenv("MSCCL_AMD_FUSE", raising=False)
    with CoResident(2, [xmlgen.allreduce_pair_oneshot(4, "LL"), xmlgen.allreduce_allpairs(2, 2, "LL")],
                    str(tmp_path)) as cr:
        for c in cr.comms:
            assert c.info()["algoFuse"] == [[0, 1, 2, 3], []], c.info()["algoFuse"]
    monkeypatch.setenv("MSCCL_AMD_FUSE", "0")
    with CoResident(2, [xmlgen.allreduce_pair_oneshot(4, "LL")], str(tmp_path)) as cr:
        assert all(c.info()["algoFuse"] == [[]] for c in cr.comms)


# counts: one pack per lane and less, one FIFO step per workgroup, several steps per pass (the
# pipeline's steady state: 1 << 20 with one instance is 4 steps in each of 4 passes), a call that
# is not whole packs (split 1, element tails), the bench's 4 and 32 MiB points
@pytest.mark.parametrize("inst,count,dt,op", [
    (1, 32, 7, 0), (1, 3000, 7, 0), (1, 1 << 16, 7, 0), (1, 1 << 20, 7, 0), (16, 1 << 20, 7, 0),
    (16, 1 << 23, 7, 0),
    (4, 1 << 18, 6, 0), (4, 1 << 18, 9, 0), (2, 100003 * 2, 6, 2), (4, 1 << 18, 2, 1), (1, 12345, 0, 0),
    (2, 1 << 17, 8, 3),
])
def test_fused_matches_oracle_and_unfused(inst, count, dt, op, tmp_path, monkeypatch):
    xml = xmlgen.allreduce_pair_oneshot(inst, "LL")
    res = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("MSCCL_AMD_FUSE", fuse)
        got, want, _ = run_collective(xml, 2, L.ALLREDUCE, count, dt, op, True, seed=4, tmpdir=str(tmp_path))
        _check(got, want, "fuse=%s" % fuse)
        res[fuse] = got
    _check(res["1"], res["0"], "fused vs unfused")


@pytest.mark.parametrize("count", [4096, 1 << 18])
def test_fused_out_of_place(count, tmp_path):
    xml = xmlgen.allreduce_pair_oneshot(4, "LL", inplace=False)
    got, want, _ = run_collective(xml, 2, L.ALLREDUCE, count, 7, 0, False, seed=8, tmpdir=str(tmp_path))
    _check(got, want, "out of place")


def test_fused_across_ll_cleanup(tmp_path, monkeypatch):
    """MSCCL_AMD_TEST_LL_CLEANUP (8-bit flags, cleanup 8 steps in every 128): 24 launches of 16
    fused FIFO steps per workgroup cross the flag wrap and several cleanup steps; Max is
    idempotent, so the repeated in-place result stays the oracle's."""
    monkeypatch.setenv("MSCCL_AMD_TEST_LL_CLEANUP", "1")
    xml = xmlgen.allreduce_pair_oneshot(1, "LL")
    got, want, _ = run_collective(xml, 2, L.ALLREDUCE, 1 << 20, 7, 2, True, seed=6, iters=24,
                                  tmpdir=str(tmp_path))
    _check(got, want, "cleanup")


def _asymmetric_xml() -> str:
    """2 ranks, one chunk: rank 0 sends then receives (a fusable shape), rank 1 receives, reduces
    and only then sends.  Run fused on rank 0 alone, a call of more than one FIFO step would
    deadlock (rank 0 waits for a step rank 1 sends only after receiving all of rank 0's)."""
    gpus = {}
    t0 = _Tb(0, 1, 1, 0)
    t0.add("s", "i", 0, "i", 0, 1)
    t0.add("rrc", "i", 0, "i", 0, 1)
    gpus[0] = (1, 0, 0, [t0])
    t1 = _Tb(0, 0, 0, 0)
    t1.add("rrc", "i", 0, "i", 0, 1)
    t1.add("s", "i", 0, "i", 0, 1)
    gpus[1] = (1, 0, 0, [t1])
    return _emit("asym", "LL", 1, 1, 2, "allreduce", True, gpus, 0, 1 << 40, None)


def test_asymmetric_exchange_is_not_fused(tmp_path):
    xml = _asymmetric_xml()
    with CoResident(2, [xml], str(tmp_path)) as cr:
        assert all(c.info()["algoFuse"] == [[]] for c in cr.comms)
    got, want, _ = run_collective(xml, 2, L.ALLREDUCE, 1 << 21, 7, 0, True, seed=2, tmpdir=str(tmp_path))
    _check(got, want, "asymmetric")


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
    for _ in range(3):
        comm.all_reduce(t.data_ptr(), t.data_ptr(), count, M.FLOAT32, M.SUM, s)
    torch.cuda.synchronize()
    info = comm.info()
    out = t.cpu().numpy()
    err = comm.async_error()
    comm.destroy()
    q_out.put((rank, err, info["last"]["small"], info["algoFuse"], out))


def test_fused_rank_interoperates_with_unfused_rank(tmp_path):
    """Rank 0 runs mscclSmallKernel (fused exchange), rank 1 the general kernel (s, then rrc):
    several FIFO steps per call, the values are the oracle's."""
    import torch.multiprocessing as mp
    from oracle import plan as P, sim as S
    world, count = 2, 1 << 20
    xml = xmlgen.allreduce_pair_oneshot(1, "LL")
    p = tmp_path / "pair.xml"
    p.write_text(xml)
    ctx = mp.get_context("spawn")
    q_in, q_out = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=_mixed_proc, args=(r, world, str(p), count, "1" if r == 0 else "0", q_in, q_out))
          for r in range(world)]
    for pr in ps:
        pr.start()
    res = {}
    for _ in range(world):
        r, err, small, fuse, out = q_out.get(timeout=300)
        res[r] = (err, small, fuse, out)
    for pr in ps:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert res[0][1] == 1 and res[1][1] == 0, (res[0][1], res[1][1])
    assert res[0][2] == [[0]] and res[1][2] == [[0]]
    algos = [L.parse_xml(xml, r, world) for r in range(world)]
    call = P.Call(L.ALLREDUCE, count, 7, 0, world, 0, True)
    plan = P.make_plan([algos[0]], call, 0)
    ins = gen_inputs(world, count, 7, 9)
    for _ in range(3):
        ins, _st = S.run(algos, plan, ins, [None] * world, L.ALLREDUCE, True)
    for r in range(world):
        assert res[r][0] == 0
        assert np.array_equal(res[r][3].view(np.uint32), np.asarray(ins[r]).view(np.uint32))


@pytest.mark.parametrize("proto,count,dt", [("LL128", 1 << 18, 7), ("LL128", 3000, 6), ("Simple", 1 << 20, 9),
                                            ("Simple", 12345, 7)])
def test_fusable_image_on_other_protocols(proto, count, dt, tmp_path):
    """The pair exchange's image carries the fused transfer type whatever the protocol; LL128 and
    Simple run it as its s followed by its rrc, with the oracle's values."""
    xml = xmlgen.allreduce_pair_oneshot(4 if count % 4 == 0 else 1, proto)
    with CoResident(2, [xml], str(tmp_path)) as cr:
        assert all(len(c.info()["algoFuse"][0]) > 0 for c in cr.comms)
    got, want, _ = run_collective(xml, 2, L.ALLREDUCE, count, dt, 0, True, seed=12, tmpdir=str(tmp_path))
    _check(got, want, proto)


@pytest.mark.parametrize("n,proto,count,dt", [(2, "Simple", 1 << 20, 7), (2, "LL", 3000, 6), (4, "Simple", 12345, 9),
                                              (8, "LL", 1 << 16, 7), (2, "LL128", 1 << 18, 2)])
def test_allgather_send_copy_fused(n, proto, count, dt, tmp_path, monkeypatch):
    """Out-of-place AllGather: the own block's cpy follows the first peer's s of the same chunk and
    the two run as one copy-send (transport.cc: kSendCopy); same bytes as unfused, oracle values."""
    xml = xmlgen.allgather_allpairs(n, 2, proto, inplace=False)
    res = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("MSCCL_AMD_FUSE", fuse)
        got, want, _ = run_collective(xml, n, L.ALLGATHER, count, dt, 0, False, seed=21, tmpdir=str(tmp_path))
        _check(got, want, "AllGather fuse=%s" % fuse)
        res[fuse] = got
    _check(res["1"], res["0"], "AllGather fused vs unfused")


# ---------------------------------------------------------------------------------------------
# The pair kernel (interpreter.h: PairRunner): a pair-form schedule (every thread block one fused
# s + rrc of affine chunks, transport.cc: pair form) whose call is one pass runs without the
# image interpreter.  Same FIFO steps as the small kernel, so the values must be the oracle's and
# bit-identical to MSCCL_AMD_PAIR_KERNEL=0's.
@pytest.mark.parametrize("inst,count,dt,op,inplace", [
    (1, 2048, 7, 0, True), (1, 3000, 7, 0, True), (16, 1 << 18, 7, 0, True), (16, 1 << 20, 9, 0, True),
    (4, 1 << 16, 6, 2, True), (2, 10003 * 2, 6, 1, True), (4, 1 << 16, 2, 3, True), (1, 12345, 0, 0, True),
    (16, 1 << 19, 8, 0, True), (4, 1 << 14, 7, 0, False), (16, 77776, 9, 2, False),
])
def test_pair_kernel_matches_oracle_and_small_kernel(inst, count, dt, op, inplace, tmp_path, monkeypatch):
    xml = xmlgen.allreduce_pair_oneshot(inst, "LL", inplace=inplace)
    monkeypatch.setenv("MSCCL_AMD_LOWER_MAX_BYTES", "0")
    res = {}
    for pk in ("1", "0"):
        monkeypatch.setenv("MSCCL_AMD_PAIR_KERNEL", pk)
        got, want, _ = run_collective(xml, 2, L.ALLREDUCE, count, dt, op, inplace, seed=31, tmpdir=str(tmp_path))
        last = run_collective.last
        assert all(l["small"] == 1 and l["pair"] == (pk == "1") for l in last), last
        _check(got, want, "pair kernel=%s" % pk)
        res[pk] = got
    _check(res["1"], res["0"], "pair vs small kernel")


def test_pair_kernel_across_ll_cleanup(tmp_path, monkeypatch):
    """24 pair-kernel launches across the 8-bit flag wrap and its cleanup steps (as
    test_fused_across_ll_cleanup); Max keeps the in-place result the oracle's."""
    monkeypatch.setenv("MSCCL_AMD_TEST_LL_CLEANUP", "1")
    monkeypatch.setenv("MSCCL_AMD_LOWER_MAX_BYTES", "0")
    xml = xmlgen.allreduce_pair_oneshot(16, "LL")
    got, want, _ = run_collective(xml, 2, L.ALLREDUCE, 1 << 18, 7, 2, True, seed=6, iters=24,
                                  tmpdir=str(tmp_path))
    assert all(l["pair"] == 1 for l in run_collective.last), run_collective.last
    _check(got, want, "pair kernel cleanup")


def test_pair_kernel_leaves_multi_pass_calls_to_other_kernels(tmp_path, monkeypatch):
    """A call of more than one pass (1 instance, 4 MiB) keeps the general kernel."""
    monkeypatch.setenv("MSCCL_AMD_LOWER_MAX_BYTES", "0")
    xml = xmlgen.allreduce_pair_oneshot(1, "LL")
    got, want, _ = run_collective(xml, 2, L.ALLREDUCE, 1 << 20, 7, 0, True, seed=3, tmpdir=str(tmp_path))
    assert all(l["pair"] == 0 for l in run_collective.last), run_collective.last
    _check(got, want, "multi-pass")


def _pair_mixed_proc(rank, world, xml_path, count, env, q_in, q_out):
    import torch
    os.environ["MSCCL_XML_FILES"] = xml_path
    os.environ["MSCCL_AMD_TIMEOUT_SEC"] = "30"
    os.environ["MSCCL_AMD_LOWER_MAX_BYTES"] = "0"
    os.environ.update(env)
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
    for _ in range(3):
        comm.all_reduce(t.data_ptr(), t.data_ptr(), count, M.FLOAT32, M.SUM, s)
    torch.cuda.synchronize()
    info = comm.info()
    out = t.cpu().numpy()
    err = comm.async_error()
    comm.destroy()
    q_out.put((rank, err, info["last"]["small"], info["last"].get("pair", 0), out))


@pytest.mark.parametrize("count", [1 << 18, 1 << 23])
@pytest.mark.parametrize("peer", ["general", "small"])
def test_pair_kernel_interoperates_with_other_kernels(peer, count, tmp_path):
    """Rank 0 runs the pair kernel, rank 1 the general kernel or the small kernel's fused exchange:
    one pass of 16 thread blocks (32 MiB: 64 iterations merged into it on both ranks, whatever
    kernel each runs), three calls, the oracle's values."""
    import torch.multiprocessing as mp
    from oracle import plan as P, sim as S
    world = 2
    xml = xmlgen.allreduce_pair_oneshot(16, "LL")
    p = tmp_path / "pair16.xml"
    p.write_text(xml)
    env1 = {"MSCCL_AMD_SMALL_KERNEL": "0"} if peer == "general" else {"MSCCL_AMD_PAIR_KERNEL": "0"}
    ctx = mp.get_context("spawn")
    q_in, q_out = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=_pair_mixed_proc, args=(r, world, str(p), count, {} if r == 0 else env1, q_in, q_out))
          for r in range(world)]
    for pr in ps:
        pr.start()
    res = {}
    for _ in range(world):
        r, err, small, pair, out = q_out.get(timeout=300)
        res[r] = (err, small, pair, out)
    for pr in ps:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert res[0][2] == 1 and res[1][2] == 0, (res[0], res[1])
    assert res[1][1] == (0 if peer == "general" else 1)
    algos = [L.parse_xml(xml, r, world) for r in range(world)]
    call = P.Call(L.ALLREDUCE, count, 7, 0, world, 0, True)
    plan = P.make_plan([algos[0]], call, 0)
    ins = gen_inputs(world, count, 7, 9)
    for _ in range(3):
        ins, _st = S.run(algos, plan, ins, [None] * world, L.ALLREDUCE, True)
    for r in range(world):
        assert res[r][0] == 0
        assert np.array_equal(res[r][3].view(np.uint32), np.asarray(ins[r]).view(np.uint32))


@pytest.mark.parametrize("nbytes", [128, 4092, 8192, 1 << 20, 32 << 20])
def test_c2_tiers_take_the_pair_kernel(nbytes, tmp_path, monkeypatch):
    """The pair one-shot tiers (bench.PAIR_TIERS, C2's tiers in rounds 2-5) with default settings:
    every one-pass size runs the pair kernel (small calls included: the pair form is not lowered by
    default), the oracle's values."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    monkeypatch.delenv("MSCCL_AMD_LOWER_MAX_BYTES", raising=False)
    tiers = bench.make_xmls(2, "LL", 16, str(tmp_path), bench.PAIR_TIERS)
    path = [t[3] for t in tiers if t[0] <= nbytes < t[1]][0]
    got, want, _ = run_collective(open(path).read(), 2, L.ALLREDUCE, nbytes // 4, 7, 0, True, seed=nbytes % 91,
                                  tmpdir=str(tmp_path))
    assert all(l["pair"] == 1 and l["ringColl"] == 0 for l in run_collective.last), run_collective.last
    _check(got, want, "C2 tier %d B" % nbytes)


@pytest.mark.parametrize("nbytes", [128, 4080, 8192, 1 << 20, 32 << 20])
def test_c2_default_tiers_run_the_allpairs_xml_lowered(nbytes, tmp_path, monkeypatch):
    """bench.py's C2 tiers (the msccl-tools two-phase all-pairs XML): calls up to 4 KiB run the
    one-hop fold, larger ones the pair exchange on the flat connections, with the values of the
    schedule as written (oracle/sim.py runs the XML)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    monkeypatch.delenv("MSCCL_AMD_LOWER_MAX_BYTES", raising=False)
    monkeypatch.delenv("MSCCL_AMD_LOWER_LARGE", raising=False)   # (this module's fixture sets it to 0)
    tiers = bench.make_xmls(2, "LL", 16, str(tmp_path))
    path = [t[3] for t in tiers if t[0] <= nbytes < t[1]][0]
    got, want, _ = run_collective(open(path).read(), 2, L.ALLREDUCE, nbytes // 4, 7, 0, True, seed=nbytes % 83,
                                  tmpdir=str(tmp_path))
    kernel = 2 if nbytes <= 4096 else 3
    assert all(l["kernel"] == kernel and l["ringColl"] == 5 for l in run_collective.last), run_collective.last
    _check(got, want, "C2 all-pairs tier %d B" % nbytes)


def test_pair_tiers_long_mixed_sequence(tmp_path):
    """C2's tiers through a long sequence of launches whose sizes jump between the pair kernel
    (one pass), the small kernel's merged passes (64 MiB, more than 64 iterations) and back, in
    one communicator pair: the FIFO steps, flags and epochs carried from launch to launch must stay
    aligned.  Exact-integer inputs; every call is checked against the exact sum."""
    import torch
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    tiers = bench.make_xmls(2, "LL", 16, str(tmp_path), bench.PAIR_TIERS)
    os.environ["MSCCL_XML_FILES"] = ":".join(t[3] for t in tiers)
    comms = M.Comm.init_all([0, 0])
    try:
        dev = torch.device("cuda:0")
        maxc = (64 << 20) // 4
        base = [torch.randint(-4, 5, (maxc,), device=dev, dtype=torch.int32).float() for _ in range(2)]
        want_full = base[0] + base[1]
        bufs = [torch.empty(maxc, device=dev) for _ in range(2)]
        s = torch.cuda.current_stream().cuda_stream
        sizes = [128, 32 << 20, 4096, 64 << 20, 1 << 20, 8192, 64 << 20, 32 << 20, 128, 16 << 20]
        kinds = []
        for rep in range(3):
            for nb in sizes:
                cnt = nb // 4
                for _ in range(4):
                    for b, x in zip(bufs, base):
                        b[:cnt].copy_(x[:cnt])
                    with M.group():
                        for c, b in zip(comms, bufs):
                            c.all_reduce(b.data_ptr(), b.data_ptr(), cnt, M.FLOAT32, M.SUM, s)
                torch.cuda.synchronize()
                assert all(c.async_error() == 0 for c in comms)
                for b in bufs:
                    assert torch.equal(b[:cnt], want_full[:cnt]), "size %d rep %d" % (nb, rep)
                last = comms[0].info()["last"]
                kinds.append((nb, last.get("pair", 0), last["small"]))
        assert (32 << 20, 1, 1) in kinds and (64 << 20, 0, 1) in kinds, kinds
    finally:
        for c in comms:
            c.destroy()


def test_pair_merge_bound_with_small_fifo_and_general_peer(tmp_path):
    """A pair-form call's merged run of sends stays within the FIFO whatever its slot size: with
    NCCL_LL_BUFFSIZE=256 KiB (32-KiB slots) a 32 MiB call is 16 slots per workgroup, so it runs as
    two passes of 8; rank 1 runs the general kernel, which sends its whole run before receiving
    (a one-pass cut would deadlock against rank 0's pair of runs).  The oracle's values."""
    import torch.multiprocessing as mp
    from oracle import plan as P, sim as S
    world, count = 2, 1 << 23
    xml = xmlgen.allreduce_pair_oneshot(16, "LL")
    p = tmp_path / "pair16.xml"
    p.write_text(xml)
    small_fifo = {"NCCL_LL_BUFFSIZE": str(256 << 10)}
    envs = [dict(small_fifo), dict(small_fifo, MSCCL_AMD_SMALL_KERNEL="0")]
    ctx = mp.get_context("spawn")
    q_in, q_out = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=_pair_mixed_proc, args=(r, world, str(p), count, envs[r], q_in, q_out))
          for r in range(world)]
    for pr in ps:
        pr.start()
    res = {}
    for _ in range(world):
        r, err, small, pair, out = q_out.get(timeout=300)
        res[r] = (err, small, pair, out)
    for pr in ps:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert res[1][1] == 0, res[1][:3]
    algos = [L.parse_xml(xml, r, world) for r in range(world)]
    call = P.Call(L.ALLREDUCE, count, 7, 0, world, 0, True)
    plan = P.make_plan([algos[0]], call, 0)
    ins = gen_inputs(world, count, 7, 9)
    for _ in range(3):
        ins, _st = S.run(algos, plan, ins, [None] * world, L.ALLREDUCE, True)
    for r in range(world):
        assert res[r][0] == 0
        assert np.array_equal(res[r][3].view(np.uint32), np.asarray(ins[r]).view(np.uint32))

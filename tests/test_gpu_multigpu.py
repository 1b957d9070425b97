"""Ranks on different GPUs: the cross-GPU branches of the transport and of the primitives.

On one MI355X every other GPU test runs its ranks co-resident on cuda:0.  The branches that only a
second device reaches are tested here, and skip (with the reason) when fewer than two devices are
visible:
  * ncclCommInitAll over distinct devices: peer access and peer FIFO pointers
    (reference init.cc:428-439, transport/p2p.cc:250-297);
  * one process per GPU: FIFOs mapped with hipIpc between devices (init.cc:271-278,
    p2p.cc:143-163,315-331);
  * the system-scope release before a Simple tail towards another GPU and the receiver's
    system-scope acquire (interpreter.h: simpleOp / waitRecvTail; prims_simple.h:218);
  * LL128 towards a remote peer (runs as LL unless MSCCL_AMD_LL128_REMOTE=1) and the 16-B line
    atomicity probe that gates it;
  * bench.py's xGMI calibration.
Every collective is compared bit for bit with the oracle (oracle/sim.py).  The probe itself also
runs on one device (writer and reader on cuda:0), so the machinery is exercised on any box.
"""
import os

import numpy as np
import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from oracle import loader as L

pytestmark = pytest.mark.gpu
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "20")


def _ndev():
    import torch
    return torch.cuda.device_count()


needs2 = pytest.mark.skipif("_ndev() < 2", reason="needs two visible GPUs (cross-GPU transport)")


def _bits(a):
    a = np.ascontiguousarray(a)
    return a.view({1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[a.dtype.itemsize])


def _check(gpu, ora, what):
    from tests.gpu_harness import describe_mismatch
    for r, (g, o) in enumerate(zip(gpu, ora)):
        assert np.array_equal(_bits(g), _bits(o)), "%s rank %d:\n%s" % (what, r, describe_mismatch(g, o))


# ------------------------------------------------------------------------------------------------
# one process, two devices (ncclCommInitAll([0, 1]))

@needs2
@pytest.mark.parametrize("proto", ["LL", "Simple", "LL128"])
@pytest.mark.parametrize("nbytes", [4096, 1 << 20, 32 << 20])
def test_init_all_two_devices_allreduce(proto, nbytes):
    from tests.gpu_harness import run_collective
    xml = xmlgen.allreduce_allpairs(2, 4, proto)
    gpu, ora, _ = run_collective(xml, 2, L.ALLREDUCE, nbytes // 4, 7, 0, True, seed=11, devices=[0, 1])
    _check(gpu, ora, "AllReduce %s %d B" % (proto, nbytes))


@needs2
@pytest.mark.parametrize("proto", ["LL", "Simple"])
def test_init_all_two_devices_pair_exchange_fp16(proto):
    """The bench's 2-rank schedule (s + rrc, fused in the small kernel) across devices."""
    from tests.gpu_harness import run_collective
    xml = xmlgen.allreduce_pair_oneshot(16, proto)
    gpu, ora, _ = run_collective(xml, 2, L.ALLREDUCE, (8 << 20) // 2, 6, 0, True, seed=12, devices=[0, 1])
    _check(gpu, ora, "pair exchange %s" % proto)


@needs2
@pytest.mark.parametrize("proto", ["LL", "Simple"])
def test_init_all_two_devices_rs_ag(proto):
    from tests.gpu_harness import run_collective
    rs = xmlgen.reduce_scatter_allpairs(2, 4, proto)
    gpu, ora, _ = run_collective(rs, 2, L.REDUCE_SCATTER, 1 << 18, 7, 0, False, seed=13, devices=[0, 1])
    _check(gpu, ora, "ReduceScatter %s" % proto)
    ag = xmlgen.allgather_allpairs(2, 4, proto)
    gpu, ora, _ = run_collective(ag, 2, L.ALLGATHER, 1 << 18, 7, 0, False, seed=14, devices=[0, 1])
    _check(gpu, ora, "AllGather %s" % proto)


@pytest.mark.skipif("_ndev() < 4", reason="needs four visible GPUs")
def test_init_all_four_devices_two_ranks_each():
    """8 ranks on 4 devices: co-resident pairs plus cross-device peers in one schedule."""
    from tests.gpu_harness import run_collective
    xml = xmlgen.allreduce_allpairs(8, 1, "LL")
    gpu, ora, _ = run_collective(xml, 8, L.ALLREDUCE, 1 << 16, 6, 0, True, seed=15,
                                 devices=[0, 0, 1, 1, 2, 2, 3, 3])
    _check(gpu, ora, "8 ranks on 4 devices")


@needs2
def test_ll128_remote_parity_many_launches(monkeypatch):
    """LL128 towards another GPU with MSCCL_AMD_LL128_REMOTE=1: many launches, bit-exact (a torn
    16-B line would hand the receiver a stale payload under a new flag)."""
    from tests.gpu_harness import run_collective
    monkeypatch.setenv("MSCCL_AMD_LL128_REMOTE", "1")
    xml = xmlgen.allreduce_allpairs(2, 8, "LL128")
    gpu, ora, _ = run_collective(xml, 2, L.ALLREDUCE, (4 << 20) // 2, 6, 0, True, seed=16, iters=50,
                                 mode="exact", devices=[0, 1])
    _check(gpu, ora, "LL128 remote")


# ------------------------------------------------------------------------------------------------
# one process per device (hipIpc between GPUs)

def _rank_proc(rank, world, xml_path, count, dt, iters, q_in, q_out):
    import torch
    os.environ["MSCCL_XML_FILES"] = xml_path
    os.environ["MSCCL_AMD_TIMEOUT_SEC"] = "30"
    torch.cuda.set_device(rank)
    uid = M.get_unique_id() if rank == 0 else None
    if rank == 0:
        for _ in range(world - 1):
            q_in.put(uid)
    else:
        uid = q_in.get(timeout=60)
    from tests.gpu_harness import gen_inputs, to_torch
    x = gen_inputs(world, count, dt, 21)[rank]
    comm = M.Comm.init_rank(world, uid, rank)
    t = to_torch(x, torch.device("cuda", rank))
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(iters):
        comm.all_reduce(t.data_ptr(), t.data_ptr(), count, dt, M.SUM, s)
    torch.cuda.synchronize()
    err = comm.async_error()
    dev = comm.device
    out = t.cpu().numpy()
    comm.destroy()
    q_out.put((rank, err, dev, out))


@needs2
@pytest.mark.parametrize("proto", ["LL", "Simple"])
def test_two_processes_two_devices_ipc(tmp_path, proto):
    import torch.multiprocessing as mp
    from tests.gpu_harness import gen_inputs
    from oracle import plan as P, sim as S
    world, count, dt, iters = 2, 1 << 20, 7, 3
    xml = xmlgen.allreduce_allpairs(world, 4, proto)
    p = tmp_path / "ap.xml"
    p.write_text(xml)
    ctx = mp.get_context("spawn")
    q_in, q_out = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=_rank_proc, args=(r, world, str(p), count, dt, iters, q_in, q_out)) for r in range(world)]
    for pr in ps:
        pr.start()
    res = {}
    for _ in range(world):
        r, err, dev, out = q_out.get(timeout=300)
        res[r] = (err, dev, out)
    for pr in ps:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    algos = [L.parse_xml(xml, r, world) for r in range(world)]
    call = P.Call(L.ALLREDUCE, count, dt, 0, world, 0, True)
    plan = P.make_plan([algos[0]], call, 0)
    ins = gen_inputs(world, count, dt, 21)
    for _ in range(iters):
        ins, _st = S.run(algos, plan, ins, [None] * world, L.ALLREDUCE, True)
    for r in range(world):
        assert res[r][0] == 0 and res[r][1] == r
        assert np.array_equal(res[r][2].view(np.uint32), np.asarray(ins[r]).view(np.uint32))


# ------------------------------------------------------------------------------------------------
# line atomicity probe and xGMI calibration

def test_line_tear_probe_local():
    """The probe's machinery on one device: lines written and polled in cuda:0's uncached memory
    are never seen torn, and every reader sees the last iteration."""
    r = M.line_tear_probe(0, 0, lines=1 << 14, iters=200, seconds=5.0)
    assert r["torn"] == 0, r
    assert r["done"] == r["lines"], r
    assert r["seen"] >= r["lines"], r


@needs2
def test_line_tear_probe_across_devices():
    """The LL128-over-xGMI gate: 16-B lines stored from cuda:0 into cuda:1's FIFO
    memory while cuda:1 polls them; a torn line fails the gate."""
    r = M.line_tear_probe(0, 1, lines=1 << 16, iters=2000, seconds=10.0)
    print("line tear probe 0 -> 1:", r)
    assert r["done"] == r["lines"], r
    assert r["torn"] == 0, r
    r = M.line_tear_probe(1, 0, lines=1 << 16, iters=2000, seconds=10.0)
    print("line tear probe 1 -> 0:", r)
    assert r["torn"] == 0, r


@needs2
def test_calibrate_xgmi_returns_a_rate():
    import sys
    sys.argv, argv = ["bench.py"], sys.argv
    try:
        import bench
    finally:
        sys.argv = argv
    gbs = bench.calibrate_xgmi(nbytes=64 << 20, reps=3)
    print("one-way peer copy cuda:0 -> cuda:1: %s GB/s" % gbs)
    assert isinstance(gbs, float) and gbs > 1.0

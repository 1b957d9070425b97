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


# ------------------------------------------------------------------------------------------------
# eight devices: BASELINE.json's 8-GPU configs (C3, C4, C5), one rank per GPU.  They run on the
# first 8-GPU box (the driver's round-end node); on fewer devices they skip with the reason.

needs8 = pytest.mark.skipif("_ndev() < 8", reason="needs eight visible GPUs (C3 / C4 / C5, one rank per GPU)")


def _bench():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    import bench
    return bench


def _c3_xml(tmp_path, nbytes):
    b = _bench()
    tiers = b.make_xmls(8, "LL", 8, str(tmp_path), remote=True)
    return open(b.tier_of(tiers, nbytes)[3]).read()


@needs8
@pytest.mark.parametrize("nbytes", [128, 64 << 10, 256 << 10, 32 << 20])
def test_c3_init_all_eight_devices(tmp_path, nbytes):
    """C3 (8 ranks, LL, fp16) through ncclCommInitAll(0..7) and bench.py's tier schedule of the size
    for ranks on different GPUs: peer pointers over xGMI to all 7 peers, bit-exact against the
    oracle (256 KiB: lowered to the fold by the link model's limit, plan.cc)."""
    from tests.gpu_harness import run_collective
    gpu, ora, _ = run_collective(_c3_xml(tmp_path, nbytes), 8, L.ALLREDUCE, nbytes // 2, 6, 0, True, seed=31,
                                 devices=list(range(8)))
    _check(gpu, ora, "C3 %d B on 8 devices" % nbytes)


@needs8
def test_c4_init_all_eight_devices():
    """C4 (8 ranks, ring, Simple, bf16, 32 rings over the 7 Hamiltonian cycles): the oracle at 8 MiB
    per rank, exact integers at the full 256 MiB (every association order gives the exact sum)."""
    from tests.gpu_harness import run_collective
    xml = xmlgen.allreduce_ring(8, 32, "Simple", True, 0, 1 << 40, name="c4_ring")
    gpu, ora, _ = run_collective(xml, 8, L.ALLREDUCE, (8 << 20) // 2, 9, 0, True, seed=32, devices=list(range(8)))
    _check(gpu, ora, "C4 8 MiB on 8 devices")
    gpu, ora, _ = run_collective(xml, 8, L.ALLREDUCE, (256 << 20) // 2, 9, 0, True, seed=33, mode="exact",
                                 devices=list(range(8)))
    _check(gpu, ora, "C4 256 MiB exact on 8 devices")


@needs8
def test_c5_init_all_eight_devices():
    """C5 (8 ranks, fp32, 64 MiB): ReduceScatter (chain form) then AllGather, Simple, each bit-exact."""
    from tests.gpu_harness import run_collective
    rc = (64 << 20) // 4 // 8
    rs = xmlgen.reduce_scatter_allpairs(8, 4, "Simple", False, 0, 1 << 40, name="c5_rs")
    gpu, ora, _ = run_collective(rs, 8, L.REDUCE_SCATTER, rc, 7, 0, False, seed=34, devices=list(range(8)))
    _check(gpu, ora, "C5 ReduceScatter on 8 devices")
    ag = xmlgen.allgather_allpairs(8, 4, "Simple", False, 0, 1 << 40, name="c5_ag")
    gpu, ora, _ = run_collective(ag, 8, L.ALLGATHER, rc, 7, 0, False, seed=35, devices=list(range(8)))
    _check(gpu, ora, "C5 AllGather on 8 devices")


def _rank_proc8(rank, world, xml_path, jobs, q_in, q_out, one_gpu=False, env=None):
    """One rank of a one-process-per-rank job: every (coll, count, dt, seed) of `jobs` in place
    (AllReduce) or out of place (RS / AG), results back to the parent.  one_gpu: every process on
    cuda:0 (hipIpc FIFOs between processes of one GPU), else rank r on cuda:r."""
    import torch
    os.environ["MSCCL_XML_FILES"] = xml_path
    os.environ["MSCCL_AMD_TIMEOUT_SEC"] = "60"
    os.environ.update(env or {})
    torch.cuda.set_device(0 if one_gpu else rank)
    uid = M.get_unique_id() if rank == 0 else None
    if rank == 0:
        for _ in range(world - 1):
            q_in.put(uid)
    else:
        uid = q_in.get(timeout=120)
    from tests.gpu_harness import gen_inputs, to_torch
    comm = M.Comm.init_rank(world, uid, rank)
    dev = torch.device("cuda", 0 if one_gpu else rank)
    s = torch.cuda.current_stream().cuda_stream
    outs = []
    kernels = []
    for coll, count, dt, seed in jobs:
        if coll == L.ALLREDUCE:
            t = to_torch(gen_inputs(world, count, dt, seed)[rank], dev)
            comm.all_reduce(t.data_ptr(), t.data_ptr(), count, dt, M.SUM, s)
        elif coll == L.REDUCE_SCATTER:
            x = to_torch(gen_inputs(world, count * world, dt, seed)[rank], dev)
            t = torch.zeros(count, dtype=x.dtype, device=dev)
            comm.reduce_scatter(x.data_ptr(), t.data_ptr(), count, dt, M.SUM, s)
        else:
            x = to_torch(gen_inputs(world, count, dt, seed)[rank], dev)
            t = torch.zeros(count * world, dtype=x.dtype, device=dev)
            comm.all_gather(x.data_ptr(), t.data_ptr(), count, dt, s)
        torch.cuda.synchronize()
        outs.append(t.cpu().numpy())
        last = comm.info()["last"]
        kernels.append(last["kernel"])  # 0 general, 1 small, 2 fold, 3 pair, 4 two-phase kernel
    err = comm.async_error()
    remote = comm.info()["anyRemote"]
    comm.destroy()
    q_out.put((rank, err, outs, kernels, remote))


def _eight_processes(tmp_path, xmls, jobs, world=8, one_gpu=False, env=None):
    """`world` rank processes (8 by default), results {rank: (async error, outputs, kernels, anyRemote)}."""
    import torch.multiprocessing as mp
    paths = []
    for i, x in enumerate(xmls):
        p = tmp_path / ("s%d.xml" % i)
        p.write_text(x)
        paths.append(str(p))
    ctx = mp.get_context("spawn")
    q_in, q_out = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=_rank_proc8, args=(r, world, ":".join(paths), jobs, q_in, q_out, one_gpu, env))
          for r in range(world)]
    for pr in ps:
        pr.start()
    res = {}
    for _ in range(world):
        r, err, outs, kernels, remote = q_out.get(timeout=600)
        res[r] = (err, outs, kernels, remote)
    for pr in ps:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    return res


def _oracle(xmls, coll, count, dt, seed, in_place, world=8):
    """The oracle's outputs of one call of the job (the schedule the reference's selection picks
    among xmls, tests/gpu_harness.py: CoResident.oracle without a GPU)."""
    import types
    from tests.gpu_harness import CoResident, gen_inputs
    fake = types.SimpleNamespace(n=world, algos=[[L.parse_xml(x, r, world) for x in xmls] for r in range(world)])
    n_in = count * world if coll == L.REDUCE_SCATTER else count
    outs, _ = CoResident.oracle(fake, coll, count, dt, 0, gen_inputs(world, n_in, dt, seed), in_place)
    return outs


def _c3_c5_job(tmp_path, remote):
    """bench.py's 8-rank C3 tiers (fp16; one rank per GPU: the remote tiers) at 128 B, 64 KiB,
    256 KiB and 32 MiB, then C5's ReduceScatter and AllGather (fp32, 64 MiB, bench.py's 8
    instances)."""
    b = _bench()
    tiers = b.make_xmls(8, "LL", 8, str(tmp_path), remote=remote)
    c3 = [open(t[3]).read() for t in tiers]
    rc = (64 << 20) // 4 // 8
    c5 = [xmlgen.reduce_scatter_allpairs(8, 8, "Simple", False, 0, 1 << 40, name="c5_rs"),
          xmlgen.allgather_allpairs(8, 8, "Simple", False, 0, 1 << 40, name="c5_ag")]
    jobs = [(L.ALLREDUCE, nb // 2, 6, 40 + k) for k, nb in enumerate((128, 64 << 10, 256 << 10, 32 << 20))]
    jobs += [(L.REDUCE_SCATTER, rc, 7, 50), (L.ALLGATHER, rc, 7, 51)]
    return c3, c5, jobs


def _check_c3_c5(res, c3, c5, jobs):
    for j, (coll, count, dt, seed) in enumerate(jobs):
        xs = c3 if coll == L.ALLREDUCE else c5
        want = _oracle(xs, coll, count, dt, seed, coll == L.ALLREDUCE)
        for r in range(8):
            assert res[r][0] == 0
            _check([res[r][1][j]], [want[r]], "8 processes job %d rank %d" % (j, r))


@needs8
def test_eight_processes_c3_c5_ipc(tmp_path):
    """One process per GPU (the reference's mpirun -np 8 -g 1, README.md:57): hipIpc FIFOs between
    all 8 GPUs, C3's remote tiers (256 KiB lowered to the fold by the link model, 32 MiB to the
    two-phase fold), then C5's
    ReduceScatter and AllGather, every rank bit-exact against the oracle."""
    c3, c5, jobs = _c3_c5_job(tmp_path, True)
    res = _eight_processes(tmp_path, c3 + c5, jobs)
    _check_c3_c5(res, c3, c5, jobs)
    assert all(res[r][3] == 1 for r in range(8))
    assert [res[0][2][j] for j in range(4)] == [2, 2, 2, 4]  # fold up to 256 KiB, then the two-phase fold


def test_eight_processes_one_gpu_c3_c5_ipc(tmp_path):
    """The driver's 8-process configuration on one GPU (bench.py --gpus 8 with
    MSCCL_AMD_BENCH_ONE_GPU=1): 8 rank processes on cuda:0, FIFOs mapped with hipIpc between
    processes, bench.py's 8-rank C3 tiers and C5's pair at full size, every rank bit-exact against
    the oracle.  Runs on any box (the needs8 form above takes the same jobs across 8 GPUs)."""
    c3, c5, jobs = _c3_c5_job(tmp_path, False)
    res = _eight_processes(tmp_path, c3 + c5, jobs, one_gpu=True)
    _check_c3_c5(res, c3, c5, jobs)
    assert all(res[r][3] == 0 for r in range(8))
    assert [res[0][2][j] for j in range(4)] == [2, 2, 4, 4]  # co-resident: fold up to 128 KiB, then two-phase


def test_eight_processes_one_gpu_forced_remote(tmp_path):
    """The driver's 8-GPU configuration as closely as one GPU allows: 8 rank processes, bench.py's
    cross-GPU tiers (8 all-pairs instances from 64 KiB, the fold up to the link model's 256 KiB)
    and the runtime's cross-GPU paths (MSCCL_AMD_FORCE_REMOTE=1: every peer treated as remote, so
    the system-scope Simple release / acquire, LL128 as LL, the remote lowering limit), C3's sizes
    and C5's pair, every rank bit-exact against the oracle."""
    c3, c5, jobs = _c3_c5_job(tmp_path, True)
    res = _eight_processes(tmp_path, c3 + c5, jobs, one_gpu=True, env={"MSCCL_AMD_FORCE_REMOTE": "1"})
    _check_c3_c5(res, c3, c5, jobs)
    assert all(res[r][3] == 1 for r in range(8))
    assert [res[0][2][j] for j in range(4)] == [2, 2, 2, 4]  # the remote limit: the fold at 256 KiB


def _c4_job():
    xml = xmlgen.allreduce_ring(8, 32, "Simple", True, 0, 1 << 40, name="c4_ring")
    return xml, [(L.ALLREDUCE, (8 << 20) // 2, 9, 60)]


@needs8
def test_eight_processes_c4_ipc(tmp_path):
    """C4 one rank per GPU: the 32-ring Simple bf16 schedule at 8 MiB per rank against the oracle."""
    xml, jobs = _c4_job()
    res = _eight_processes(tmp_path, [xml], jobs)
    want = _oracle([xml], L.ALLREDUCE, (8 << 20) // 2, 9, 60, True)
    for r in range(8):
        assert res[r][0] == 0
        _check([res[r][1][0]], [want[r]], "C4 8 processes rank %d" % r)


def test_eight_processes_one_gpu_c4_ipc(tmp_path):
    """C4's 32-ring Simple bf16 schedule, 8 rank processes on cuda:0 (hipIpc), 8 MiB per rank,
    bit-exact against the oracle."""
    xml, jobs = _c4_job()
    res = _eight_processes(tmp_path, [xml], jobs, one_gpu=True)
    want = _oracle([xml], L.ALLREDUCE, (8 << 20) // 2, 9, 60, True)
    for r in range(8):
        assert res[r][0] == 0
        _check([res[r][1][0]], [want[r]], "C4 8 processes on one GPU rank %d" % r)


# ------------------------------------------------------------------------------------------------
# four devices: bench.py --gpus 4 (fp32, one rank per GPU, the 4-rank remote tiers)

needs4 = pytest.mark.skipif("_ndev() < 4", reason="needs four visible GPUs (bench.py --gpus 4, one rank per GPU)")


def _four_rank_job(tmp_path, remote):
    b = _bench()
    tiers = b.make_xmls(4, "LL", 8, str(tmp_path), remote=remote)
    xmls = [open(t[3]).read() for t in tiers]
    jobs = [(L.ALLREDUCE, nb // 4, 7, 70 + k) for k, nb in enumerate((128, 64 << 10, 256 << 10, 4 << 20, 32 << 20))]
    return xmls, jobs


def _check_four(res, xmls, jobs):
    for j, (coll, count, dt, seed) in enumerate(jobs):
        want = _oracle(xmls, coll, count, dt, seed, True, world=4)
        for r in range(4):
            assert res[r][0] == 0
            _check([res[r][1][j]], [want[r]], "4 processes job %d rank %d" % (j, r))


@needs4
def test_four_processes_four_devices_bench_tiers(tmp_path):
    """bench.py --gpus 4: 4 rank processes on 4 GPUs (hipIpc over xGMI), the 4-rank remote tiers
    (one-shot below 64 KiB, two-phase all-pairs above, fold up to the link model's 256 KiB), fp32,
    128 B to 32 MiB, bit-exact against the oracle."""
    xmls, jobs = _four_rank_job(tmp_path, True)
    res = _eight_processes(tmp_path, xmls, jobs, world=4)
    _check_four(res, xmls, jobs)
    assert all(res[r][3] == 1 for r in range(4))
    assert [res[0][2][j] for j in range(3)] == [2, 2, 2]


def test_four_processes_one_gpu_bench_tiers(tmp_path):
    """The same 4-rank job with the 4 processes on cuda:0 (co-resident tiers and limits)."""
    xmls, jobs = _four_rank_job(tmp_path, False)
    res = _eight_processes(tmp_path, xmls, jobs, world=4, one_gpu=True)
    _check_four(res, xmls, jobs)
    assert [res[0][2][j] for j in range(3)] == [2, 2, 4]


# ------------------------------------------------------------------------------------------------
# two ranks: bench.py --gpus 2 (C2: fp32, one rank per GPU, the all-pairs XML tiers)

def _two_rank_job(tmp_path, remote):
    b = _bench()
    tiers = b.make_xmls(2, "LL", 16, str(tmp_path), remote=remote)
    xmls = [open(t[3]).read() for t in tiers]
    sizes = (128, 4096, 8192, 1 << 20, 32 << 20)
    return xmls, [(L.ALLREDUCE, nb // 4, 7, 80 + k) for k, nb in enumerate(sizes)]


def _check_two(res, xmls, jobs):
    for j, (coll, count, dt, seed) in enumerate(jobs):
        want = _oracle(xmls, coll, count, dt, seed, True, world=2)
        for r in range(2):
            assert res[r][0] == 0
            _check([res[r][1][j]], [want[r]], "2 processes job %d rank %d" % (j, r))


@needs2
def test_two_processes_two_devices_c2_tiers(tmp_path):
    """bench.py --gpus 2: 2 rank processes on 2 GPUs (hipIpc over xGMI), C2's tiers 128 B - 32 MiB
    (the two-phase all-pairs XML, lowered): the fold up to 4 KiB, the pair kernel on the flat
    connections above, bit-exact against the oracle running the XML."""
    xmls, jobs = _two_rank_job(tmp_path, True)
    res = _eight_processes(tmp_path, xmls, jobs, world=2)
    _check_two(res, xmls, jobs)
    assert all(res[r][3] == 1 for r in range(2))
    assert res[0][2] == [2, 2, 3, 3, 3], res[0][2]


def test_two_processes_one_gpu_forced_remote_c2_tiers(tmp_path):
    """The same job with both processes on cuda:0 and every peer treated as remote
    (MSCCL_AMD_FORCE_REMOTE=1: the cross-GPU limits and paths the N=2 driver run takes)."""
    xmls, jobs = _two_rank_job(tmp_path, True)
    res = _eight_processes(tmp_path, xmls, jobs, world=2, one_gpu=True, env={"MSCCL_AMD_FORCE_REMOTE": "1"})
    _check_two(res, xmls, jobs)
    assert all(res[r][3] == 1 for r in range(2))
    assert res[0][2] == [2, 2, 3, 3, 3], res[0][2]

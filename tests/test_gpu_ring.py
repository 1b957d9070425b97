"""GPU parity of the ring fallback (no MSCCL schedule matches, enqueue.cc:461-476): the HIP
interpreter's ring mode vs oracle/ring.py (a restatement of the reference's runRing,
all_reduce.h:14-100, reduce_scatter.h:13-67, all_gather.h:13-78), bit-exact, on co-resident ranks.
Sizes are chosen ragged: not multiples of any chunk, channel or rank count."""
import os

import numpy as np
import pytest

import msccl_amd as M
from oracle import loader as L
from tests.gpu_harness import gen_inputs, to_torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _ring_algorithm(monkeypatch):
    """These cases pin the ring (small AllReduces take the tree by default: plan.cc makeRingPlan);
    the tree tests select it themselves."""
    monkeypatch.setenv("NCCL_ALGO", "Ring,Tree")
    monkeypatch.setenv("MSCCL_AMD_TREE_MAX_BYTES", "0")
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "20")


def check(n, coll, count, dt, op=0, in_place=True, seed=3, iters=1, user_scale=None):
    from tests.gpu_harness import run_ring_fallback
    gpu, ora, rp = run_ring_fallback(n, coll, count, dt, op, in_place, seed, iters=iters, user_scale=user_scale)
    for r in range(n):
        g, o = gpu[r].view(np.uint8), ora[r].view(np.uint8)
        if not np.array_equal(g, o):
            bad = np.nonzero(g != o)[0]
            raise AssertionError("rank %d (%r): %d differing bytes, first at %d" % (r, rp, len(bad), bad[0]))
    return rp


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("count", [1, 37, 4099, 100003, 1234567])
@pytest.mark.parametrize("dt", [7, 6, 9])
def test_ring_allreduce(n, count, dt):
    check(n, L.ALLREDUCE, count, dt)    # LL up to 512 KiB, Simple above


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("count", [1, 333, 40001, 300007])
@pytest.mark.parametrize("in_place", [True, False])
def test_ring_reduce_scatter(n, count, in_place):
    check(n, L.REDUCE_SCATTER, count, 7, in_place=in_place)


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("count", [1, 333, 40001, 300007])
@pytest.mark.parametrize("in_place", [True, False])
def test_ring_all_gather(n, count, in_place):
    check(n, L.ALLGATHER, count, 6, in_place=in_place)


@pytest.mark.parametrize("op", [1, 2, 3])
def test_ring_ops_out_of_place(op):
    check(4, L.ALLREDUCE, 77777, 7, op=op, in_place=False)


def test_ring_repeated_launches_and_integers():
    check(4, L.ALLREDUCE, 5000, 2, iters=12)
    check(3, L.ALLREDUCE, 300001, 4, iters=3)


def test_ring_channels_forced(monkeypatch):
    monkeypatch.setenv("MSCCL_AMD_RING_CHANNELS", "3")
    rp = check(4, L.ALLREDUCE, 654321, 9)
    assert rp["channels"] == 3


@pytest.mark.parametrize("name", ["fb3_ring_ar_f32", "fb4_ring_rs_bf16", "fb2_ring_ag_f16", "fb8_ring_ar_f16_max"])
def test_ring_golden_vectors_on_gpu(name):
    from tests.golden import make_golden as G
    from tests.gpu_harness import run_ring_fallback
    _, n, coll, count, dt, op, inplace = [c for c in G.RING_CASES if c[0] == name][0]
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name + ".npz"))
    gpu, _, _ = run_ring_fallback(n, coll, count, dt, op, inplace, seed=7)
    for r in range(n):
        assert np.array_equal(gpu[r].view(np.uint8), z["outputs"][r].view(np.uint8)), r


# ---- ncclAvg and user PreMulSum ops (enqueue.cc:1388-1454, 1529-1580; reduce_kernel.h:498-687):
# MSCCL never takes them (tuning.cc:345), the ring does: inputs scaled before the sum (floats) or
# the sum divided after (integers).  LL sizes and Simple sizes, every element type.
@pytest.mark.parametrize("dt", [7, 6, 9, 8, 2, 3, 0, 1, 4, 5])
@pytest.mark.parametrize("count", [4099, 300001])
def test_ring_avg_allreduce(dt, count):
    check(3, L.ALLREDUCE, count, dt, op=4, in_place=True)


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("dt", [7, 9, 2])
def test_ring_avg_allreduce_ranks_and_out_of_place(n, dt):
    check(n, L.ALLREDUCE, 77777, dt, op=4, in_place=False)


@pytest.mark.parametrize("dt", [7, 6, 2, 5])
@pytest.mark.parametrize("in_place", [True, False])
def test_ring_avg_reduce_scatter(dt, in_place):
    check(4, L.REDUCE_SCATTER, 40001, dt, op=4, in_place=in_place)
    check(4, L.REDUCE_SCATTER, 300007, dt, op=4, in_place=in_place)


@pytest.mark.parametrize("dt,value", [(7, 0.37), (6, -1.75), (9, 3.0), (8, 0.1), (2, 3), (1, 7)])
@pytest.mark.parametrize("residence", [1, 0])
def test_ring_user_premulsum(dt, value, residence):
    """ncclRedOpCreatePreMulSum with the scale in host memory (read at creation) or in device
    memory (read by the kernel)."""
    check(4, L.ALLREDUCE, 12345, dt, user_scale=(value, residence))
    check(3, L.ALLREDUCE, 400001, dt, user_scale=(value, residence))


def test_avg_one_rank_and_user_op_one_rank():
    """nRanks == 1: ncclAvg is a copy (enqueue.cc:811-816), a user PreMulSum still scales the data
    (oneRankReduce, onerank_reduce.cu:12-44), in place and out of place."""
    import torch
    import msccl_amd as M
    from oracle import numerics as N
    comm = M.Comm.init_all([0])[0]
    try:
        x = torch.randn(100003, device="cuda")
        y = torch.zeros_like(x)
        s = torch.cuda.current_stream().cuda_stream
        comm.all_reduce(x.data_ptr(), y.data_ptr(), x.numel(), M.FLOAT32, M.AVG, s)
        torch.cuda.synchronize()
        assert torch.equal(x, y)
        op = comm.create_premulsum(np.float32(0.3).tobytes(), M.FLOAT32, M.SCALAR_HOST)
        comm.all_reduce(x.data_ptr(), y.data_ptr(), x.numel(), M.FLOAT32, op, s)
        z = x.clone()
        comm.all_reduce(z.data_ptr(), z.data_ptr(), z.numel(), M.FLOAT32, op, s)
        torch.cuda.synchronize()
        want = N.pre_op(N.PREMULSUM, 7, x.cpu().numpy(), N.scalar_bits(7, 0.3))
        assert np.array_equal(y.cpu().numpy().view(np.uint32), want.view(np.uint32))
        assert np.array_equal(z.cpu().numpy().view(np.uint32), want.view(np.uint32))
        comm.destroy_op(op)
    finally:
        comm.destroy()


def test_user_op_errors():
    """Builtin or unknown ops cannot be destroyed; a destroyed op, or one created on another
    communicator or for another type, is rejected (enqueue.cc:1388-1454, 1563-1580)."""
    import torch
    import msccl_amd as M
    comms = M.Comm.init_all([0, 0])
    try:
        x = torch.zeros(1024, device="cuda")
        with pytest.raises(M.NcclError):
            comms[0].destroy_op(M.SUM)
        op0 = comms[0].create_premulsum(np.float32(2).tobytes(), M.FLOAT32)
        op1 = comms[1].create_premulsum(np.float32(2).tobytes(), M.FLOAT32)
        assert op0 >= 5 and op1 >= 5
        if op0 != op1:   # mangled with the communicator: op0 means nothing to comms[1]
            with pytest.raises(M.NcclError):
                comms[1].all_reduce(x.data_ptr(), x.data_ptr(), 1024, M.FLOAT32, op0, 0)
        with pytest.raises(M.NcclError):   # type mismatch
            comms[0].all_reduce(x.data_ptr(), x.data_ptr(), 512, M.FLOAT16, op0, 0)
        comms[0].destroy_op(op0)
        with pytest.raises(M.NcclError):
            comms[0].destroy_op(op0)
        with pytest.raises(M.NcclError):
            comms[0].all_reduce(x.data_ptr(), x.data_ptr(), 1024, M.FLOAT32, op0, 0)
        comms[1].destroy_op(op1)
    finally:
        for c in comms:
            c.destroy()


# ---- tree fallback (all_reduce.h:103-298 on a chain, NCCL_ALGO=Tree) -----------------------------
@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("count", [1, 37, 4099, 100003, 1234567])
@pytest.mark.parametrize("dt", [7, 6, 9])
def test_tree_allreduce(monkeypatch, n, count, dt):
    monkeypatch.setenv("NCCL_ALGO", "Tree")
    rp = check(n, L.ALLREDUCE, count, dt)
    assert rp["algo"] == "tree"


@pytest.mark.parametrize("op", [1, 2, 3, 4])
@pytest.mark.parametrize("dt", [7, 2])
def test_tree_ops_out_of_place_and_avg(monkeypatch, op, dt):
    monkeypatch.setenv("NCCL_ALGO", "Tree")
    check(4, L.ALLREDUCE, 77777, dt, op=op, in_place=False)
    check(4, L.ALLREDUCE, 777777, dt, op=op, in_place=True)


def test_tree_threshold_and_repeats(monkeypatch):
    """MSCCL_AMD_TREE_MAX_BYTES routes small AllReduces to the tree and larger ones to the ring on
    the same communicators; repeated launches keep both connection sets in step."""
    monkeypatch.setenv("MSCCL_AMD_TREE_MAX_BYTES", str(64 << 10))
    assert check(4, L.ALLREDUCE, 5000, 7, iters=5)["algo"] == "tree"
    monkeypatch.delenv("MSCCL_AMD_TREE_MAX_BYTES")        # default: the LL range for the flat tree
    assert check(4, L.ALLREDUCE, 131072, 7)["last"]["ringColl"] == 5
    assert check(4, L.ALLREDUCE, 131073, 7)["algo"] == "ring"
    assert check(4, L.ALLREDUCE, 50000, 7, iters=2)["last"]["ringColl"] == 5
    assert check(4, L.ALLREDUCE, 16384, 7, op=4)["algo"] == "tree"   # Avg: 16 KiB per rank
    assert check(4, L.ALLREDUCE, 16385, 7, op=4)["algo"] == "ring"
    monkeypatch.setenv("MSCCL_AMD_TREE_FLAT", "0")         # without the flat tree: 16 KiB per rank
    assert check(4, L.ALLREDUCE, 16384, 7)["algo"] == "tree"
    assert check(4, L.ALLREDUCE, 16385, 7)["algo"] == "ring"


# ---- flat tree: the chain tree's values in one hop (plan.cc: makeFlatTreePlan) -------------------
def _flat_env(monkeypatch, tree_max=None):
    monkeypatch.setenv("NCCL_ALGO", "Ring,Tree")
    if tree_max is None:
        # defaults: AllReduce up to 512 KiB on the flat tree; flat ReduceScatter / AllGather over
        # the whole LL range (512 KiB in all), no per-block cap
        monkeypatch.delenv("MSCCL_AMD_TREE_MAX_BYTES", raising=False)
    else:
        monkeypatch.setenv("MSCCL_AMD_TREE_MAX_BYTES", str(tree_max))


@pytest.mark.parametrize("n", [2, 3, 4, 8, 16])
@pytest.mark.parametrize("count", [1, 37, 511, 512, 4099])
@pytest.mark.parametrize("dt", [7, 6, 9])
def test_flat_tree_equals_the_chain_tree(monkeypatch, n, count, dt):
    """Small AllReduces take the flat tree (every rank sends its input to every peer and folds the
    n inputs in the chain's order x_{n-1} (+) ... (+) x_0, one hop) in the fold kernel
    ("small" 2, interpreter.h: runFold); the oracle is oracle/ring.py's chain tree."""
    _flat_env(monkeypatch)
    rp = check(n, L.ALLREDUCE, count, dt, seed=5 + n)
    assert rp["algo"] == "tree"
    assert rp["last"]["ringColl"] == 5 and rp["last"]["small"] == 2, rp["last"]


@pytest.mark.parametrize("op,dt", [(1, 7), (2, 6), (3, 9), (0, 2), (1, 4), (2, 0)])
@pytest.mark.parametrize("in_place", [True, False])
def test_flat_tree_ops(monkeypatch, op, dt, in_place):
    _flat_env(monkeypatch)
    rp = check(4, L.ALLREDUCE, 3001, dt, op=op, in_place=in_place, iters=3)
    assert rp["last"]["ringColl"] == 5, rp["last"]


def test_flat_tree_multi_iteration_and_chain_knob(monkeypatch):
    """Several FIFO steps per call (8192 floats a step, a ragged last one), repeated launches;
    MSCCL_AMD_TREE_FLAT=0 keeps the chain; Avg (PreMulSum) always takes the chain."""
    _flat_env(monkeypatch, 256 << 10)
    rp = check(8, L.ALLREDUCE, 50001, 7, iters=2)
    assert rp["last"]["ringColl"] == 5, rp["last"]
    rp = check(8, L.ALLREDUCE, 8192 * 4, 7)
    assert rp["last"]["ringColl"] == 5 and rp["last"]["small"] == 2, rp["last"]
    assert check(4, L.ALLREDUCE, 3001, 7, op=4)["last"]["ringColl"] == 4
    monkeypatch.setenv("MSCCL_AMD_TREE_FLAT", "0")
    rp = check(8, L.ALLREDUCE, 4099, 6)
    assert rp["algo"] == "tree" and rp["last"]["ringColl"] == 4, rp["last"]


def test_flat_tree_across_ll_cleanup(monkeypatch):
    """MSCCL_AMD_TEST_LL_CLEANUP=1 (8-bit flags, cleanup 8 steps in every 128): 300 fold-kernel
    launches cross the flag wrap and the cleanup steps on every connection (the fold kernel stamps
    its send slots' unused lines itself); Max is idempotent, so the in-place result stays the
    chain tree's."""
    _flat_env(monkeypatch)
    monkeypatch.setenv("MSCCL_AMD_TEST_LL_CLEANUP", "1")
    rp = check(4, L.ALLREDUCE, 4099, 6, op=2, iters=300)
    assert rp["last"]["ringColl"] == 5 and rp["last"]["small"] == 2, rp["last"]


@pytest.mark.parametrize("n", [2, 3, 4, 8, 16])
@pytest.mark.parametrize("count", [1, 37, 512, 4095])
@pytest.mark.parametrize("in_place", [True, False])
def test_flat_reduce_scatter_equals_the_ring(monkeypatch, n, count, in_place):
    """LL ReduceScatters in the LL range (no per-block cap by default; MSCCL_AMD_TREE_MAX_BYTES caps a
    rank's block when set) take the fold kernel's one hop: block
    p to peer p, the own block folded in the ring's order x_{r+1} (+) ... (+) x_{r+n-1} (+) x_r;
    the oracle is oracle/ring.py's ring (reduce_scatter.h:13-67), bit for bit."""
    _flat_env(monkeypatch)
    rp = check(n, L.REDUCE_SCATTER, count, 7, in_place=in_place, seed=7 + n)
    assert rp["last"]["ringColl"] == 5 and rp["last"]["small"] == 2, rp["last"]


@pytest.mark.parametrize("n", [2, 3, 4, 8, 16])
@pytest.mark.parametrize("count", [1, 37, 512, 8191])
@pytest.mark.parametrize("in_place", [True, False])
def test_flat_all_gather_equals_the_ring(monkeypatch, n, count, in_place):
    """LL AllGathers in the LL range (no per-block cap by default) take the fold kernel: every rank's
    block to every
    peer, each stored at its place (all_gather.h:13-78's result)."""
    _flat_env(monkeypatch)
    rp = check(n, L.ALLGATHER, count, 6, in_place=in_place, seed=9 + n)
    assert rp["last"]["ringColl"] == 5 and rp["last"]["small"] == 2, rp["last"]


@pytest.mark.parametrize("op,dt", [(1, 6), (2, 9), (3, 2), (0, 8), (2, 0)])
def test_flat_reduce_scatter_ops_and_limits(monkeypatch, op, dt):
    """Ops Sum..Min on other types, repeated launches; a block over the limit takes the ring, and
    Avg (PreMulSum) always does."""
    _flat_env(monkeypatch)
    rp = check(4, L.REDUCE_SCATTER, 1001, dt, op=op, in_place=False, iters=3)
    assert rp["last"]["ringColl"] == 5, rp["last"]
    _flat_env(monkeypatch, 512)
    rp = check(4, L.REDUCE_SCATTER, 1001, dt, op=op)
    assert rp["last"]["ringColl"] == 2, rp["last"]
    _flat_env(monkeypatch)
    assert check(4, L.REDUCE_SCATTER, 1001, 7, op=4)["last"]["ringColl"] == 2
    monkeypatch.setenv("MSCCL_AMD_TREE_FLAT", "0")
    assert check(4, L.ALLGATHER, 1001, 7)["last"]["ringColl"] == 3


def test_flat_all_gather_across_ll_cleanup(monkeypatch):
    """300 in-place AllGathers across the 8-bit flag wrap and cleanup steps."""
    _flat_env(monkeypatch)
    monkeypatch.setenv("MSCCL_AMD_TEST_LL_CLEANUP", "1")
    rp = check(3, L.ALLGATHER, 2047, 0, iters=300)
    assert rp["last"]["ringColl"] == 5 and rp["last"]["small"] == 2, rp["last"]


def _flat_proc(rank, world, count, q_in, q_out):
    import torch
    os.environ.pop("MSCCL_XML_FILES", None)
    os.environ["NCCL_ALGO"] = "Ring,Tree"
    os.environ["MSCCL_AMD_TIMEOUT_SEC"] = "30"
    torch.cuda.set_device(0)
    uid = M.get_unique_id() if rank == 0 else None
    if rank == 0:
        for _ in range(world - 1):
            q_in.put(uid)
    else:
        uid = q_in.get(timeout=60)
    x = gen_inputs(world, count, 7, 13)[rank]
    comm = M.Comm.init_rank(world, uid, rank)
    t = to_torch(x, torch.device("cuda:0"))
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(4):
        comm.all_reduce(t.data_ptr(), t.data_ptr(), count, M.FLOAT32, M.SUM, s)
    torch.cuda.synchronize()
    err = comm.async_error()
    last = comm.info()["last"]
    out = t.cpu().numpy()
    comm.destroy()
    q_out.put((rank, err, last["ringColl"], last["small"], out))


def test_flat_tree_across_processes(monkeypatch):
    """One rank per process (hipIpc FIFOs): each process launches its own fold kernel; the values
    are the chain tree's (oracle/ring.py), 4 in-place AllReduces in a row."""
    import torch.multiprocessing as mp
    from oracle import ring as R
    _flat_env(monkeypatch)   # inherited by the spawned ranks
    world, count = 3, 1001
    ctx = mp.get_context("spawn")
    q_in, q_out = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=_flat_proc, args=(r, world, count, q_in, q_out)) for r in range(world)]
    for pr in ps:
        pr.start()
    res = {}
    for _ in range(world):
        r, err, ring_coll, small, out = q_out.get(timeout=300)
        res[r] = (err, ring_coll, small, out)
    for pr in ps:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    ins = gen_inputs(world, count, 7, 13)
    for _ in range(4):
        ins, _rp = R.run(L.ALLREDUCE, count, 7, 0, ins, [None] * world, True, 0)
    for r in range(world):
        assert res[r][0] == 0 and res[r][1] == 5 and res[r][2] == 2, res[r][:3]
        assert np.array_equal(res[r][3].view(np.uint32), np.asarray(ins[r]).view(np.uint32))


@pytest.mark.parametrize("n,coll,count,dt,in_place", [
    (8, L.ALLREDUCE, (512 << 10) // 2, 6, True), (8, L.ALLREDUCE, 2049, 9, False), (3, L.ALLREDUCE, 4099, 7, True),
    (8, L.REDUCE_SCATTER, 4097, 7, False), (4, L.REDUCE_SCATTER, 333, 7, True),
    (8, L.ALLGATHER, 8001, 6, False), (2, L.ALLGATHER, 333, 6, True)])
def test_ring_one_iteration_small_kernel(monkeypatch, n, coll, count, dt, in_place):
    """LL ring calls whose runRing loop covers the call once run mscclSmallKernel's ring pass
    (enqueue.cc: smallEligible, profiles/r05p_ring_small_ab.txt: 8 ranks 512 KiB 72.4 -> 62.6 us),
    bit-exact against oracle/ring.py; MSCCL_AMD_SMALL_KERNEL=0 keeps the general kernel, same bits."""
    monkeypatch.setenv("MSCCL_AMD_TREE_FLAT", "0")   # the ring itself, not its one-hop flat form
    rp = check(n, coll, count, dt, in_place=in_place, seed=count % 17)
    assert rp["last"]["ringColl"] in (1, 2, 3) and rp["last"]["proto"] == 0 and rp["last"]["small"] == 1, rp
    monkeypatch.setenv("MSCCL_AMD_SMALL_KERNEL", "0")
    rp = check(n, coll, count, dt, in_place=in_place, seed=count % 17)
    assert rp["last"]["small"] == 0, rp


def test_ring_multi_iteration_keeps_general_kernel(monkeypatch):
    """A call the ring loop covers more than once stays in the general kernel."""
    monkeypatch.setenv("MSCCL_AMD_TREE_FLAT", "0")
    rp = check(2, L.ALLREDUCE, (512 << 10) // 2, 6)
    assert rp["last"]["small"] == 0 and rp["last"]["proto"] == 0, rp

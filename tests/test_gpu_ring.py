"""GPU parity of the ring fallback (no MSCCL schedule matches, enqueue.cc:461-476): the HIP
interpreter's ring mode vs oracle/ring.py (a restatement of the reference's runRing,
all_reduce.h:14-100, reduce_scatter.h:13-67, all_gather.h:13-78), bit-exact, on co-resident ranks.
Sizes are chosen ragged: not multiples of any chunk, channel or rank count."""
import os

import numpy as np
import pytest

from oracle import loader as L

pytestmark = pytest.mark.gpu
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "20")


def check(n, coll, count, dt, op=0, in_place=True, seed=3, iters=1):
    from tests.gpu_harness import run_ring_fallback
    gpu, ora, rp = run_ring_fallback(n, coll, count, dt, op, in_place, seed, iters=iters)
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

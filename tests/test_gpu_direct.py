"""The direct form of Simple schedules on the GPU (lower.h: DirectLowering, interpreter.h:
DirectRunner, enqueue.cc: launchGroup).

When every rank of a communicator is in one launch (ncclCommInitAll on one GPU, one group call),
a Simple AllGather / ReduceScatter / AllReduce call runs mscclDirectKernel (comm info last.kernel
5): every rank reads the others' buffers and writes into them, no FIFO (the reference's P2P
direct mode, prims_simple.h:75-128).  Every result is compared bit for bit with oracle/sim.py
running the XML as written (FIFOs, scratch, the schedule's fold orders)."""
import os

import numpy as np
import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from oracle import loader as L
from oracle import numerics as N
from tests.gpu_harness import CoResident, describe_mismatch, from_torch, gen_inputs, run_collective, to_torch

pytestmark = pytest.mark.gpu
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "20")

RCCL = "/opt/rocm/share/rccl/msccl-algorithms"


def _check(got, want, what):
    for r in range(len(want)):
        assert np.array_equal(np.asarray(got[r]).view(np.uint8), np.asarray(want[r]).view(np.uint8)), \
            "%s rank %d: %s" % (what, r, describe_mismatch(got[r], want[r]))


@pytest.mark.parametrize("n,inst,count,dt", [(8, 8, 1 << 18, 7), (8, 8, (1 << 18) + 4 * 8 * 8, 7), (2, 16, 1 << 20, 9),
                                            (4, 2, 3 * 1024 * 8, 6), (3, 1, 6000, 2)])
def test_reduce_scatter_and_allgather_direct(tmp_path, n, inst, count, dt):
    """C5's pair (8 ranks, x8, fp32; other rank counts and types): the ReduceScatter (chain form)
    and the AllGather run the direct kernel and give the oracle's bits."""
    rs = xmlgen.reduce_scatter_allpairs(n, inst, "Simple", False)
    got, want, _ = run_collective(rs, n, L.REDUCE_SCATTER, count, dt, 0, False, seed=count % 91, tmpdir=str(tmp_path))
    _check(got, want, "RS")
    assert all(l["kernel"] == 5 for l in run_collective.last), run_collective.last
    ag = xmlgen.allgather_allpairs(n, inst, "Simple", False)
    got, want, _ = run_collective(ag, n, L.ALLGATHER, count, dt, 0, False, seed=count % 93, tmpdir=str(tmp_path))
    _check(got, want, "AG")
    assert all(l["kernel"] == 5 for l in run_collective.last), run_collective.last


@pytest.mark.parametrize("op", [0, 1, 2, 3])
def test_reduce_scatter_scratch_form_every_op(tmp_path, op):
    rs = xmlgen.reduce_scatter_allpairs(4, 2, "Simple", False, form="scratch")
    got, want, _ = run_collective(rs, 4, L.REDUCE_SCATTER, 8 * 2048, 9, op, False, seed=op, tmpdir=str(tmp_path))
    _check(got, want, "RS scratch op %d" % op)
    assert all(l["kernel"] == 5 for l in run_collective.last), run_collective.last


@pytest.mark.parametrize("n,chans,count,dt,inplace", [(8, 32, 1 << 22, 9, True), (8, 4, 8 * 4 * 1024 * 3, 7, True),
                                                     (2, 2, 1 << 20, 6, False), (4, 8, 4 * 8 * 2048, 9, False)])
def test_ring_allreduce_direct(tmp_path, n, chans, count, dt, inplace):
    """C4's ring (8 ranks, 32 rings, Simple, bf16 8 MiB per rank) and other shapes: the direct
    kernel folds every chunk in its ring order and writes it to every rank."""
    xml = xmlgen.allreduce_ring(n, chans, "Simple", inplace, 0, 1 << 40)
    got, want, _ = run_collective(xml, n, L.ALLREDUCE, count, dt, 0, inplace, seed=count % 89, tmpdir=str(tmp_path))
    _check(got, want, "ring AR")
    assert all(l["kernel"] == 5 for l in run_collective.last), run_collective.last


def test_rccl_simple_allpairs_direct(tmp_path):
    """RCCL's shipped allreduce-allpairs-8n-simple (its `re` folds in Simple's order)."""
    p = os.path.join(RCCL, "allreduce-allpairs-8n-simple.xml")
    if not os.path.exists(p):
        pytest.skip("fixture missing")
    xml = open(p).read()
    ncpl = M.algo_json(p, 0, 8)["nchunksperloop"]
    count = ncpl * 2048
    got, want, _ = run_collective(xml, 8, L.ALLREDUCE, count, 6, 0, True, seed=4, tmpdir=str(tmp_path))
    _check(got, want, "RCCL Simple all-pairs")
    assert all(l["kernel"] == 5 for l in run_collective.last), run_collective.last


def test_small_calls_keep_the_fifo_and_interleave(tmp_path):
    """Calls below nthreads elements per chunk (Simple's per-element path) keep the interpreter;
    direct and interpreted calls alternate on one communicator set, every result bit-exact."""
    xml = xmlgen.allreduce_ring(4, 2, "Simple", True, 0, 1 << 40)
    with CoResident(4, [xml], str(tmp_path)) as cr:
        import torch
        kinds = set()
        for it in range(40):
            count = (4 * 2 * 4096, 4 * 2 * 64)[it % 2]
            ins = gen_inputs(4, count, 7, it)
            t = [to_torch(x, torch.device("cuda:0")) for x in ins]
            torch.cuda.synchronize()
            cr.run(L.ALLREDUCE, count, 7, 0, [x.data_ptr() for x in t], [x.data_ptr() for x in t])
            want, _ = cr.oracle(L.ALLREDUCE, count, 7, 0, ins, True)
            _check([from_torch(x, N.storage(7)) for x in t], want, "it %d" % it)
            kinds.add((it % 2, cr.comms[0].info()["last"]["kernel"] == 5))
        assert kinds == {(0, True), (1, False)}, kinds


def test_direct_knob_and_exact_c5_full_size(tmp_path, monkeypatch):
    """MSCCL_AMD_DIRECT=0 runs the schedule's FIFO path; both give the exact sums of C5 at its full
    size (64 MiB, 8 ranks, exact integers)."""
    rs = xmlgen.reduce_scatter_allpairs(8, 8, "Simple", False)
    ag = xmlgen.allgather_allpairs(8, 8, "Simple", False)
    rc = (64 << 20) // 4 // 8
    for direct in ("1", "0"):
        monkeypatch.setenv("MSCCL_AMD_DIRECT", direct)
        got, want, _ = run_collective(rs, 8, L.REDUCE_SCATTER, rc, 7, 0, False, seed=3, mode="exact",
                                      tmpdir=str(tmp_path))
        _check(got, want, "RS direct=%s" % direct)
        assert all((l["kernel"] == 5) == (direct == "1") for l in run_collective.last), run_collective.last
    got, want, _ = run_collective(ag, 8, L.ALLGATHER, rc, 7, 0, False, seed=5, mode="exact", tmpdir=str(tmp_path))
    _check(got, want, "AG")


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("coll,count,dt,op", [(L.REDUCE_SCATTER, 300007, 7, 0), (L.REDUCE_SCATTER, 200003, 9, 2),
                                              (L.REDUCE_SCATTER, 262147, 6, 3), (L.ALLGATHER, 300007, 6, 0),
                                              (L.ALLGATHER, 777777, 0, 0)])
@pytest.mark.parametrize("in_place", [True, False])
@pytest.mark.parametrize("direct", ["1", "0"])
def test_ring_fallback_direct(monkeypatch, n, coll, count, dt, op, in_place, direct):
    """The ring fallback's Simple ReduceScatter / AllGather (no schedule loaded, ragged sizes above
    the LL range) on ranks that share one launch: the direct form (a block folded along the ring
    from the rank after its owner; the AllGather's copies), bit-exact against oracle/ring.py's
    runRing; MSCCL_AMD_DIRECT=0 keeps the ring's FIFOs, the same bits."""
    from tests.gpu_harness import run_ring_fallback
    monkeypatch.setenv("MSCCL_AMD_DIRECT", direct)
    gpu, ora, rp = run_ring_fallback(n, coll, count, dt, op, in_place, seed=count % 97)
    assert (rp["last"]["kernel"] == 5) == (direct == "1"), rp["last"]
    for r in range(n):
        g, o = gpu[r].view(np.uint8), ora[r].view(np.uint8)
        assert np.array_equal(g, o), "rank %d: %d differing bytes" % (r, int(np.count_nonzero(g != o)))

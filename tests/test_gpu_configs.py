"""Bit-exact parity at the full size of every BASELINE.json configuration.

  C1  1 rank, fp32, 1 MiB: the nRanks == 1 copy (enqueue.cc:811-816)
  C2  2 ranks, LL, fp32, every sweep point 128 B .. 32 MiB, through bench.py's own size tiers
      (the msccl-tools two-phase all-pairs XML, x1 below 4 KiB and x16 above, lowered at upload:
      the fold up to 4 KiB, the pair exchange above)
  C3  8 ranks, LL, fp16, 128 B / 64 KiB / 1 MiB / 32 MiB: bench.py's 8-rank tiers and RCCL's
      32-tb all-pairs schedule with maxBytes raised (128 B takes the ring fallback there)
  C4  8 ranks, ring, Simple, bf16, 256 MiB per rank (bench.py's 32-ring schedule)
  C5  8 ranks, ReduceScatter then AllGather, fp32, 64 MiB total (all-pairs, Simple)

Every rank of a config runs co-resident on cuda:0 (one fused launch, local HBM in place of
xGMI).  The GPU result is compared bit for bit with the oracle (oracle/sim.py, oracle/ring.py:
the reference's association order) on seeded uniform inputs: BASELINE.md's "within 1 ulp of the
CPU reduction on the same inputs" holds with 0 ulp, the CPU reduction being the oracle's fold in
the reference's order.  Separately the result is checked against the exact sum within the
summation bound (n-1)·u·Σ|x| (for 2 ranks: the correctly rounded a+b, 0.5 ulp; for 8 ranks the
bound is wider than 1 ulp of the exact sum, which no fixed association order can promise).  C4's
256 MiB per rank is checked with exact-integer inputs at full size (every order gives the exact
sum) and against the oracle at 8 MiB per rank, which has the same iteration / merge /
maxAllowedCount structure on the device (one iteration, one-chunk transfers).
"""
import os

import numpy as np
import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from oracle import loader as L
from oracle import numerics as N
from tests.gpu_harness import CoResident, describe_mismatch, gen_inputs, sum_error_ok, to_torch, from_torch

pytestmark = pytest.mark.gpu
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "30")
RCCL = "/opt/rocm/share/rccl/msccl-algorithms"


def _bench():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    return bench


def _allreduce_case(cr: CoResident, count: int, dt: int, seed: int, label: str, ulp_bound: bool = True):
    """One in-place AllReduce on every rank of cr vs the oracle; returns the schedule used."""
    import torch
    dev = torch.device("cuda:0")
    ins = gen_inputs(cr.n, count, dt, seed)
    t = [to_torch(x, dev) for x in ins]
    torch.cuda.synchronize()
    cr.run(L.ALLREDUCE, count, dt, 0, [x.data_ptr() for x in t], [x.data_ptr() for x in t])
    gpu = [from_torch(x, N.storage(dt)) for x in t]
    want, used = cr.oracle(L.ALLREDUCE, count, dt, 0, ins, True)
    for r in range(cr.n):
        if not np.array_equal(gpu[r].view(np.uint8), want[r].view(np.uint8)):
            raise AssertionError("%s: rank %d differs from the oracle (schedule %s)\n%s" % (
                label, r, used, describe_mismatch(gpu[r], want[r])))
    if ulp_bound:
        ok, ratio = sum_error_ok(gpu[0], ins, dt)
        assert ok, "%s: error %.2f x the summation bound" % (label, ratio)
    return used


def test_c1_single_rank_copy_1mib():
    """C1: one rank, fp32, 1 MiB: out of place a device copy, in place nothing (enqueue.cc:811-816)."""
    import torch
    comm = M.Comm.init_all([0])[0]
    try:
        x = gen_inputs(1, 1 << 18, 7, 41)[0]
        a = to_torch(x, torch.device("cuda:0"))
        b = torch.full_like(a, 7.0)
        s = torch.cuda.current_stream().cuda_stream
        comm.all_reduce(a.data_ptr(), b.data_ptr(), a.numel(), M.FLOAT32, M.SUM, s)
        comm.all_reduce(a.data_ptr(), a.data_ptr(), a.numel(), M.FLOAT32, M.SUM, s)
        torch.cuda.synchronize()
        assert np.array_equal(from_torch(b, np.float32).view(np.uint32), x.view(np.uint32))
        assert np.array_equal(from_torch(a, np.float32).view(np.uint32), x.view(np.uint32))
    finally:
        comm.destroy()


def test_c2_two_ranks_ll_fp32_full_sweep(tmp_path):
    """C2: every point of bench.py's sweep through its exact tiered XMLs, twice (persistent FIFO
    state across sizes and schedules); for two ranks the result is the correctly rounded a+b."""
    b = _bench()
    tiers = b.make_xmls(2, "LL", 16, str(tmp_path))
    xmls = [open(t[3]).read() for t in tiers]
    with CoResident(2, xmls) as cr:
        for rep in range(2):
            for k, nbytes in enumerate(b.SIZES):
                count = nbytes // 4
                used = _allreduce_case(cr, count, 7, 100 * rep + k, "C2 %d B" % nbytes)
                lo, hi = tiers[used][0], tiers[used][1]
                assert lo <= nbytes < hi, (nbytes, used)


def test_c3_eight_ranks_ll_fp16_bench_tiers(tmp_path):
    """C3 with bench.py's 8-rank tiers (rank-ordered one-shot, then two-phase all-pairs)."""
    b = _bench()
    tiers = b.make_xmls(8, "LL", 4, str(tmp_path))
    xmls = [open(t[3]).read() for t in tiers]
    with CoResident(8, xmls) as cr:
        for nbytes in (128, 64 << 10, 1 << 20, 32 << 20):
            _allreduce_case(cr, nbytes // 2, 6, nbytes % 997, "C3 tiers %d B" % nbytes)


def test_c3_eight_ranks_ll_fp16_rccl_32tb():
    """C3 with RCCL's shipped 8-rank 32-tb LL all-pairs schedule, maxBytes raised to 32 MiB + 1
    (SURVEY §8(d)); 128 B (64 halves, not a multiple of nchunksperloop 256) takes the ring."""
    p = os.path.join(RCCL, "allreduce-allpairs-8n-ll-32tb.xml")
    if not os.path.exists(p):
        pytest.skip("fixture missing")
    xml = open(p).read().replace('maxBytes="65536"', 'maxBytes="%d"' % ((32 << 20) + 1))
    assert 'maxBytes="%d"' % ((32 << 20) + 1) in xml
    with CoResident(8, [xml]) as cr:
        for nbytes in (128, 64 << 10, 1 << 20, 32 << 20):
            used = _allreduce_case(cr, nbytes // 2, 6, 7 + nbytes % 991, "C3 rccl %d B" % nbytes)
            assert (used == "ring") == (nbytes == 128), (nbytes, used)


def test_c4_eight_ranks_ring_simple_bf16_256mib():
    """C4: exact-integer bf16 inputs at 256 MiB per rank (every association order gives the
    exact sum), then uniform inputs against the oracle at 8 MiB per rank."""
    import torch
    xml = xmlgen.allreduce_ring(8, 32, "Simple", True, 0, 1 << 40, name="c4_ring")
    n = 8
    with CoResident(n, [xml]) as cr:
        count = (256 << 20) // 2
        g = torch.Generator(device="cuda:0").manual_seed(4)
        bufs = [torch.randint(-4, 5, (count,), generator=g, device="cuda:0").to(torch.bfloat16) for _ in range(n)]
        want = torch.stack([x.float() for x in bufs]).sum(0).to(torch.bfloat16)
        torch.cuda.synchronize()
        cr.run(L.ALLREDUCE, count, 9, 0, [x.data_ptr() for x in bufs], [x.data_ptr() for x in bufs])
        for r in range(n):
            if not torch.equal(bufs[r], want):
                bad = (bufs[r] != want).nonzero()
                raise AssertionError("C4 256 MiB rank %d: %d elements wrong, first at %s" % (
                    r, bad.shape[0], bad[:4].flatten().tolist()))
        del bufs, want
        _allreduce_case(cr, (8 << 20) // 2, 9, 44, "C4 8 MiB uniform")


def test_c5_eight_ranks_reduce_scatter_then_allgather_fp32_64mib():
    """C5: ReduceScatter (64 MiB in, 8 MiB out per rank) then AllGather of its result, as two
    separate calls, both against the oracle at full size."""
    import torch
    n, inst = 8, 4   # 8 co-resident ranks x (8 x 4) thread blocks = 256 tbs: all resident at once
    rs = xmlgen.reduce_scatter_allpairs(n, inst, "Simple", False, 0, 1 << 40, name="c5_rs")
    ag = xmlgen.allgather_allpairs(n, inst, "Simple", False, 0, 1 << 40, name="c5_ag")
    dev = torch.device("cuda:0")
    total = (64 << 20) // 4
    rc = total // n
    with CoResident(n, [rs, ag]) as cr:
        ins = gen_inputs(n, total, 7, 55)
        t_in = [to_torch(x, dev) for x in ins]
        t_mid = [torch.zeros(rc, dtype=torch.float32, device=dev) for _ in range(n)]
        t_out = [torch.zeros(total, dtype=torch.float32, device=dev) for _ in range(n)]
        torch.cuda.synchronize()
        cr.run(L.REDUCE_SCATTER, rc, 7, 0, [x.data_ptr() for x in t_in], [x.data_ptr() for x in t_mid])
        mid = [from_torch(x, np.float32) for x in t_mid]
        want, used = cr.oracle(L.REDUCE_SCATTER, rc, 7, 0, ins, False)
        assert used == 0
        for r in range(n):
            assert np.array_equal(mid[r].view(np.uint32), want[r].view(np.uint32)), \
                "C5 RS rank %d\n%s" % (r, describe_mismatch(mid[r], want[r]))
            ok, ratio = sum_error_ok(mid[r], [x[r * rc:(r + 1) * rc] for x in ins], 7)
            assert ok, ratio
        cr.run(L.ALLGATHER, rc, 7, 0, [x.data_ptr() for x in t_mid], [x.data_ptr() for x in t_out])
        out = [from_torch(x, np.float32) for x in t_out]
        want2, used2 = cr.oracle(L.ALLGATHER, rc, 7, 0, mid, False)
        assert used2 == 1
        full = np.concatenate(mid)
        for r in range(n):
            assert np.array_equal(out[r].view(np.uint32), want2[r].view(np.uint32)), \
                "C5 AG rank %d\n%s" % (r, describe_mismatch(out[r], want2[r]))
            assert np.array_equal(out[r].view(np.uint32), full.view(np.uint32))

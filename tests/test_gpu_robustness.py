"""GPU robustness: poisoned communicators, co-residency limits, protocol selection towards remote
peers, the LL flag-cleanup path, FIFO-step agreement between the two ends of a connection, and
calls beyond a buffer descriptor's 2 GiB reach."""
import os

import numpy as np
import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from oracle import loader as L
from oracle import numerics as N
from oracle import plan as P
from oracle import sim as S
from tests.gpu_harness import CoResident, describe_mismatch, gen_inputs, to_torch, from_torch

pytestmark = pytest.mark.gpu
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "20")
RCCL = "/opt/rocm/share/rccl/msccl-algorithms"


def test_timeout_poisons_the_communicator(tmp_path):
    """A wait that times out (MSCCL_AMD_TIMEOUT_SEC) records ncclSystemError for
    ncclCommGetAsyncError, and every later collective on that communicator is refused instead of
    running on FIFO step counters that no longer match the peer's."""
    import torch
    p = tmp_path / "ap.xml"
    p.write_text(xmlgen.allreduce_allpairs(2, 1, "LL"))
    os.environ["MSCCL_XML_FILES"] = str(p)
    old = os.environ.get("MSCCL_AMD_TIMEOUT_SEC")
    os.environ["MSCCL_AMD_TIMEOUT_SEC"] = "2"
    comms = M.Comm.init_all([0, 0])
    os.environ["MSCCL_AMD_TIMEOUT_SEC"] = old or "20"
    try:
        t = torch.ones(1024, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        comms[0].all_reduce(t.data_ptr(), t.data_ptr(), 1024, M.FLOAT32, M.SUM, s)  # rank 1 never joins
        torch.cuda.synchronize()
        assert comms[0].async_error() == 2
        with pytest.raises(M.NcclError) as ei:
            comms[0].all_reduce(t.data_ptr(), t.data_ptr(), 1024, M.FLOAT32, M.SUM, s)
        assert ei.value.code == 2
        with pytest.raises(M.NcclError):
            with M.group():
                comms[0].all_reduce(t.data_ptr(), t.data_ptr(), 1024, M.FLOAT32, M.SUM, s)
    finally:
        comms[0].abort()
        comms[1].destroy()


def test_more_than_16_coresident_ranks_refused():
    """RCCL's 32-rank AllGather on one GPU: 32 co-resident ranks cannot share one launch, so
    ncclCommInitAll refuses with ncclInvalidUsage instead of launching parts that would time out."""
    p = os.path.join(RCCL, "allgather_32n_direct_0_6m_ll128.xml")
    if not os.path.exists(p):
        pytest.skip("fixture missing")
    os.environ["MSCCL_XML_FILES"] = p
    with pytest.raises(M.NcclError) as ei:
        M.Comm.init_all([0] * 32)
    assert ei.value.code == 5
    with pytest.raises(M.NcclError) as ei:
        M.Comm.init_all([0] * 17)
    assert ei.value.code == 5


def test_launch_beyond_residency_refused(tmp_path):
    """8 co-resident ranks x 128 thread blocks (16-instance all-pairs ReduceScatter) need 1,024
    workgroups resident at once, more than the GPU holds: the call fails with ncclInvalidUsage
    before launching a grid that could only hang; a 4-instance schedule runs."""
    import torch
    n = 8
    big = xmlgen.reduce_scatter_allpairs(n, 16, "Simple", False, 0, 1 << 40, name="rs16")
    with CoResident(n, [big]) as cr:
        rc = 16 * 1024
        ins = [torch.zeros(rc * n, device="cuda") for _ in range(n)]
        outs = [torch.zeros(rc, device="cuda") for _ in range(n)]
        with pytest.raises(M.NcclError) as ei:
            cr.run(L.REDUCE_SCATTER, rc, 7, 0, [x.data_ptr() for x in ins], [x.data_ptr() for x in outs])
        assert ei.value.code == 5
        assert all(c.async_error() == 0 for c in cr.comms)


@pytest.mark.parametrize("allow", [False, True])
def test_ll128_not_used_towards_remote_peers(monkeypatch, allow):
    """LL128's CDNA4 line format relies on 16-B stores arriving untorn, shown for local HBM only:
    towards peers on other GPUs (MSCCL_AMD_FORCE_REMOTE=1 here) an LL128 schedule runs with LL
    unless MSCCL_AMD_LL128_REMOTE=1.  Values are those of the reference's LL order."""
    import torch
    monkeypatch.setenv("MSCCL_AMD_FORCE_REMOTE", "1")
    if allow:
        monkeypatch.setenv("MSCCL_AMD_LL128_REMOTE", "1")
    n, count, dt = 4, 32 * 3001, 7
    xml = xmlgen.allreduce_allpairs(n, 2, "LL128")
    with CoResident(n, [xml]) as cr:
        ins = gen_inputs(n, count, dt, 12)
        t = [to_torch(x, torch.device("cuda:0")) for x in ins]
        cr.run(L.ALLREDUCE, count, dt, 0, [x.data_ptr() for x in t], [x.data_ptr() for x in t])
        info = cr.comms[0].info()
        assert info["anyRemote"] == 1
        assert info["last"]["proto"] == (L.PROTO_LL128 if allow else L.PROTO_LL)
        algos = [a[0] for a in cr.algos]
        call = P.Call(L.ALLREDUCE, count, dt, 0, n, 0, True)
        plan = P.make_plan(cr.algos[0], call, 0, proto=info["last"]["proto"])
        want, _ = S.run(algos, plan, [x.copy() for x in ins], [None] * n, L.ALLREDUCE, True)
        for r in range(n):
            got = from_torch(t[r], np.float32)
            assert np.array_equal(got.view(np.uint32), want[r].view(np.uint32)), describe_mismatch(got, want[r])


@pytest.mark.parametrize("proto", ["LL", "LL128"])
def test_ll_flag_wrap_and_cleanup(monkeypatch, proto):
    """MSCCL_AMD_TEST_LL_CLEANUP=1 is the reference's TEST_LL_CLEANUP build (devcomm.h:56-63): the
    LL flag wraps every 256 steps and senders stamp every unused line of a slot on steps with
    (step & 0x78) == 0x78 (prims_ll.h:90-97).  600 launches cross several flag wraps and
    cleanup windows; every checked launch must still produce the oracle's bits."""
    import torch
    monkeypatch.setenv("MSCCL_AMD_TEST_LL_CLEANUP", "1")
    n, dt = 2, 7
    xml = xmlgen.allreduce_allpairs(n, 2, proto, inplace=False)
    with CoResident(n, [xml]) as cr:
        dev = torch.device("cuda:0")
        sizes = [16 * 8, 16 * 1000, 16 * 4096 + 16 * 3]   # ragged: partial lines, partial slots
        wants = {}
        ins = {}
        for count in sizes:
            ins[count] = gen_inputs(n, count, dt, count % 97)
            want, used = cr.oracle(L.ALLREDUCE, count, dt, 0, ins[count], False)
            assert used == 0
            wants[count] = want
        t_in = {c: [to_torch(x, dev) for x in ins[c]] for c in sizes}
        t_out = {c: [torch.zeros(c, device=dev) for _ in range(n)] for c in sizes}
        for it in range(600):
            c = sizes[it % len(sizes)]
            cr.run(L.ALLREDUCE, c, dt, 0, [x.data_ptr() for x in t_in[c]], [x.data_ptr() for x in t_out[c]])
            if it % 37 == 0 or it >= 597:
                for r in range(n):
                    got = from_torch(t_out[c][r], np.float32)
                    assert np.array_equal(got.view(np.uint32), wants[c][r].view(np.uint32)), \
                        "launch %d count %d rank %d\n%s" % (it, c, r, describe_mismatch(got, wants[c][r]))
                    t_out[c][r].zero_()


def test_sender_and_receiver_cut_the_same_fifo_steps():
    """RCCL's 8-rank Simple all-pairs at 75 Ki floats per chunk: a `s cnt=8` call of 2.4 MB is more
    than the FIFO run bound, so the sender moves it in maxAllowedCount-sized calls of 3.4 slots;
    its receiver must cut exactly the same calls or the slots it reads would not be the ones
    written.  Bit-exact against the oracle."""
    p = os.path.join(RCCL, "allreduce-allpairs-8n-simple.xml")
    if not os.path.exists(p):
        pytest.skip("fixture missing")
    xml = open(p).read().replace('maxBytes="20971520"', 'maxBytes="%d"' % (160 << 20))
    from tests.test_gpu_configs import _allreduce_case
    with CoResident(8, [xml]) as cr:
        _allreduce_case(cr, 512 * 75 * 1024, 7, 77, "8n simple 150 MiB", ulp_bound=False)
        _allreduce_case(cr, 512 * 1000, 7, 78, "8n simple 2 MiB", ulp_bound=False)


@pytest.mark.parametrize("case", ["ring", "rccl_8n", "env"])
def test_local_simple_fifo_size(tmp_path, monkeypatch, case):
    """Ranks on one GPU take 32-KiB Simple slots (plan.h: kLocalSimpleBuff) unless a Simple
    schedule sends more than two chunks before it receives (RCCL's 8-rank all-pairs: the
    reference's 512-KiB slots) or NCCL_BUFFSIZE is set; either way the results stay bit-exact."""
    from tests.test_gpu_configs import _allreduce_case
    if case == "rccl_8n":
        p = os.path.join(RCCL, "allreduce-allpairs-8n-simple.xml")
        if not os.path.exists(p):
            pytest.skip("fixture missing")
        xml, n, want = open(p).read(), 8, 512 << 10
    else:
        xml, n, want = xmlgen.allreduce_ring(4, 4, "Simple", True, 0, 1 << 40), 4, 32 << 10
    if case == "env":
        monkeypatch.setenv("NCCL_BUFFSIZE", str(1 << 20))
        want = (1 << 20) // 8
    with CoResident(n, [xml], str(tmp_path)) as cr:
        assert all(c.info()["simpleSlotBytes"] == want for c in cr.comms)
        _allreduce_case(cr, 512 * 1024, 7, 5, "local fifo %s" % case, ulp_bound=False)


def test_calls_beyond_2gib():
    """2.4 GB per rank (600 M floats): user buffers beyond a buffer descriptor's 2 GiB reach and
    offsets beyond 2^31 elements' bytes, through an all-pairs Simple schedule and through the ring
    fallback (600 M + 1 floats matches no schedule).  Exact-integer inputs: the sum is exact."""
    import torch
    n = 2
    xml = xmlgen.allreduce_allpairs(n, 16, "Simple", True, 0, 1 << 40)
    with CoResident(n, [xml]) as cr:
        for count in (600_000_000, 600_000_001):
            g = torch.Generator(device="cuda:0").manual_seed(count % 1000)
            bufs = [torch.randint(-4, 5, (count,), generator=g, device="cuda:0").float() for _ in range(n)]
            want = bufs[0] + bufs[1]
            torch.cuda.synchronize()
            cr.run(L.ALLREDUCE, count, 7, 0, [x.data_ptr() for x in bufs], [x.data_ptr() for x in bufs])
            assert cr.comms[0].info()["last"]["ringColl"] == (0 if count % 64 == 0 else 1)
            for r in range(n):
                if not torch.equal(bufs[r], want):
                    bad = (bufs[r] != want).nonzero()
                    raise AssertionError("count %d rank %d: %d wrong, first %s" % (
                        count, r, bad.shape[0], bad[:4].flatten().tolist()))
            del bufs, want
            torch.cuda.empty_cache()


def _uneven_pair_xml(instances: int, extra: int) -> str:
    """2-rank Simple pair exchange (s, rrc per thread block) where rank 0's thread blocks first run
    `extra` local copies of their chunk into scratch: rank 0 produces late and rank 1's consumer
    spins on the tail, its previous launch's loads of the same FIFO slots still in its caches."""
    base = xmlgen.allreduce_pair_oneshot(instances, "Simple", max_bytes=1 << 24)
    out = []
    rank = None
    for line in base.splitlines():
        if line.strip().startswith("<gpu "):
            rank = int(line.split('id="')[1].split('"')[0])
            if rank == 0:
                line = line.replace('s_chunks="0"', 's_chunks="%d"' % instances)
        out.append(line)
        if rank == 0 and line.strip().startswith("<tb "):
            k = int(line.split('id="')[1].split('"')[0])
            for _ in range(extra):
                out.append('      <step s="0" type="cpy" srcbuf="i" srcoff="%d" dstbuf="s" dstoff="%d" cnt="1" '
                           'depid="-1" deps="-1" hasdep="0"/>' % (k, k))
    # renumber the steps of every thread block densely
    text, res, s = "\n".join(out), [], 0
    for line in text.splitlines():
        if line.strip().startswith("<tb "):
            s = 0
        if line.strip().startswith("<step "):
            line = line.split('s="')[0] + 's="%d"' % s + line.split('"', 2)[2][line.split('"', 2)[2].index(" "):]
            s += 1
        res.append(line)
    return "\n".join(res) + "\n"


def test_simple_handoff_uneven_load_l1_warm():
    """The unfenced local Simple hand-off (sc0 sc1 stores drained, barrier, one
    lane's tail post; the consumer polls the tail, then loads the slot after the barrier) under the
    guide's hard case: uneven load (rank 0 does extra work before every send, so rank 1 waits on
    the tail) and a consumer whose caches hold the same FIFO slots from the previous launch.  200
    launches of an int32 Sum in place (every launch changes every word, a stale word cannot repeat
    the expected value), every word of every launch checked against the oracle."""
    from tests.gpu_harness import run_collective
    xml = _uneven_pair_xml(8, 6)
    algos = [L.parse_xml(xml, r, 2) for r in range(2)]
    assert len(algos[0].tbs[0].transfers) == 8 and len(algos[1].tbs[0].transfers) == 2
    # 8 chunks of 64 Ki int32: 8 of the local 32-KiB FIFO slots per chunk (plan.h: kLocalSimpleBuff)
    gpu, ora, _ = run_collective(xml, 2, L.ALLREDUCE, 8 * (1 << 16), 2, 0, True, seed=77, iters=200)
    for r in range(2):
        assert np.array_equal(gpu[r].view(np.uint32), ora[r].view(np.uint32)), describe_mismatch(gpu[r], ora[r])

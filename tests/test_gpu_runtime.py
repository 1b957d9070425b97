"""GPU runtime behaviour: multi-process ranks over hipIpc, API edge cases, failure handling."""
import os

import numpy as np
import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from oracle import loader as L

pytestmark = pytest.mark.gpu
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "20")


def _rank_proc(rank, world, xml_path, count, q_in, q_out):
    import torch
    os.environ["MSCCL_XML_FILES"] = xml_path
    os.environ["MSCCL_AMD_TIMEOUT_SEC"] = "30"
    torch.cuda.set_device(0)
    if rank == 0:
        uid = M.get_unique_id()
        for _ in range(world - 1):
            q_in.put(uid)
    else:
        uid = None
    if uid is None:
        uid = q_in.get(timeout=60)
    from tests.gpu_harness import gen_inputs, to_torch
    x = gen_inputs(world, count, 7, 5)[rank]
    comm = M.Comm.init_rank(world, uid, rank)
    t = to_torch(x, torch.device("cuda:0"))
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        comm.all_reduce(t.data_ptr(), t.data_ptr(), count, M.FLOAT32, M.SUM, s)
    torch.cuda.synchronize()
    err = comm.async_error()
    out = t.cpu().numpy()
    comm.destroy()
    q_out.put((rank, err, out))


@pytest.mark.parametrize("proto", ["LL", "Simple"])
def test_multiprocess_ipc_ranks(tmp_path, proto):
    """Two processes, one rank each, FIFOs mapped with hipIpcOpenMemHandle (the multi-GPU path)."""
    import torch.multiprocessing as mp
    from tests.gpu_harness import gen_inputs
    from oracle import plan as P, sim as S
    world, count = 2, 16 * 4096
    xml = xmlgen.allreduce_allpairs(world, 4, proto)
    p = tmp_path / "ap.xml"
    p.write_text(xml)
    ctx = mp.get_context("spawn")
    q_in, q_out = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=_rank_proc, args=(r, world, str(p), count, q_in, q_out)) for r in range(world)]
    for pr in ps:
        pr.start()
    res = {}
    for _ in range(world):
        r, err, out = q_out.get(timeout=300)
        res[r] = (err, out)
    for pr in ps:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    algos = [L.parse_xml(xml, r, world) for r in range(world)]
    call = P.Call(L.ALLREDUCE, count, 7, 0, world, 0, True)
    plan = P.make_plan([algos[0]], call, 0)
    ins = gen_inputs(world, count, 7, 5)
    for _ in range(3):
        ins, _st = S.run(algos, plan, ins, [None] * world, L.ALLREDUCE, True)
    for r in range(world):
        assert res[r][0] == 0
        assert np.array_equal(res[r][1].view(np.uint32), np.asarray(ins[r]).view(np.uint32))


def test_single_rank_is_a_copy():
    import torch
    comm = M.Comm.init_all([0])[0]
    try:
        a = torch.randn(1 << 18, device="cuda")
        b = torch.zeros_like(a)
        s = torch.cuda.current_stream().cuda_stream
        comm.all_reduce(a.data_ptr(), b.data_ptr(), a.numel(), M.FLOAT32, M.SUM, s)   # C1: D2D copy
        comm.all_reduce(a.data_ptr(), a.data_ptr(), a.numel(), M.FLOAT32, M.SUM, s)   # in place: no-op
        torch.cuda.synchronize()
        assert torch.equal(a, b)
        assert comm.nranks == 1 and comm.rank == 0 and comm.device == 0
    finally:
        comm.destroy()


def test_no_matching_algorithm_and_zero_count(tmp_path, monkeypatch):
    """With the ring fallback disabled (MSCCL_AMD_RING_FALLBACK=0) a call no XML matches is an
    error; test_no_match_falls_back_to_ring covers the default."""
    import torch
    p = tmp_path / "ap.xml"
    p.write_text(xmlgen.allreduce_allpairs(2, 4, "LL", max_bytes=1 << 20))
    os.environ["MSCCL_XML_FILES"] = str(p)
    monkeypatch.setenv("MSCCL_AMD_RING_FALLBACK", "0")
    comms = M.Comm.init_all([0, 0])
    try:
        a = [torch.zeros(1 << 20, device="cuda") for _ in comms]
        s = torch.cuda.current_stream().cuda_stream
        with pytest.raises(M.NcclError) as ei:
            with M.group():
                for c, t in zip(comms, a):
                    c.all_reduce(t.data_ptr(), t.data_ptr(), 24, M.FLOAT32, M.SUM, s)  # 24 % 16 != 0
        assert ei.value.code == 5
        with pytest.raises(M.NcclError):
            comms[0].all_reduce(a[0].data_ptr(), a[0].data_ptr(), 1 << 19, M.FLOAT32, M.SUM, s)  # >= maxBytes
        with M.group():
            for c, t in zip(comms, a):
                c.all_reduce(t.data_ptr(), t.data_ptr(), 0, M.FLOAT32, M.SUM, s)
        torch.cuda.synchronize()
        info = comms[0].info()
        assert info["nranks"] == 2 and info["sendConns"] == 4 and info["recvConns"] == 4
    finally:
        for c in comms:
            c.destroy()


def test_no_match_falls_back_to_ring(tmp_path):
    """The reference falls back to its ring when no MSCCL algorithm matches (enqueue.cc:461-476):
    not divisible by nchunksperloop, beyond maxBytes, out of place against an in-place XML; the
    MSCCL schedule still serves the calls it matches, on the same communicators."""
    import torch
    p = tmp_path / "ap.xml"
    p.write_text(xmlgen.allreduce_allpairs(2, 4, "LL", max_bytes=1 << 20))
    os.environ["MSCCL_XML_FILES"] = str(p)
    comms = M.Comm.init_all([0, 0])
    try:
        g = torch.Generator().manual_seed(11)
        s = torch.cuda.current_stream().cuda_stream
        for count, inplace in [(24, True), (1 << 19, True), (4096, False), (4096, True), (1001, False)]:
            x = [torch.randint(-4, 5, (count,), generator=g).float() for _ in comms]
            d = [t.cuda() for t in x]
            o = d if inplace else [torch.zeros_like(t) for t in d]
            with M.group():
                for c, a, b in zip(comms, d, o):
                    c.all_reduce(a.data_ptr(), b.data_ptr(), count, M.FLOAT32, M.SUM, s)
            torch.cuda.synchronize()
            for b in o:
                assert torch.equal(b.cpu(), x[0] + x[1]), (count, inplace)
        assert all(c.async_error() == 0 for c in comms)
        # 4 all-pairs channels + 32 ring channels + 32 tree channels (rank 0 is the chain's root)
        # + the flat tree's connection to every peer (transport.cc: flatPeers)
        assert comms[0].info()["sendConns"] == 4 + 32 + 32 + 1
    finally:
        for c in comms:
            c.destroy()


def test_timeout_reports_async_error(tmp_path):
    """A rank whose peer never launches times out in-kernel and reports through ncclCommGetAsyncError."""
    import torch
    os.environ["MSCCL_AMD_TIMEOUT_SEC"] = "2"
    p = tmp_path / "ap.xml"
    p.write_text(xmlgen.allreduce_allpairs(2, 1, "LL"))
    os.environ["MSCCL_XML_FILES"] = str(p)
    comms = M.Comm.init_all([0, 0])
    os.environ["MSCCL_AMD_TIMEOUT_SEC"] = "20"
    try:
        t = torch.ones(1024, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        comms[0].all_reduce(t.data_ptr(), t.data_ptr(), 1024, M.FLOAT32, M.SUM, s)  # rank 1 never joins
        torch.cuda.synchronize()
        assert comms[0].async_error() == 2  # ncclSystemError
    finally:
        comms[0].abort()
        comms[1].destroy()


def test_stream_ordering_separate_streams():
    """Co-resident ranks issuing on different streams are fused and ordered with events."""
    import torch
    from tests.gpu_harness import gen_inputs, to_torch
    from oracle import plan as P, sim as S
    xml = xmlgen.allreduce_allpairs(2, 2, "Simple")
    path = "/tmp/msccl_streams_%d.xml" % os.getpid()
    open(path, "w").write(xml)
    os.environ["MSCCL_XML_FILES"] = path
    comms = M.Comm.init_all([0, 0])
    try:
        count = 8 * 5000
        ins = gen_inputs(2, count, 7, 9)
        dev = torch.device("cuda:0")
        ts = [to_torch(x, dev) for x in ins]
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        torch.cuda.synchronize()
        with M.group():
            for c, t, st in zip(comms, ts, streams):
                c.all_reduce(t.data_ptr(), t.data_ptr(), count, M.FLOAT32, M.SUM, st.cuda_stream)
        for st in streams:
            st.synchronize()
        algos = [L.parse_xml(xml, r, 2) for r in range(2)]
        plan = P.make_plan([algos[0]], P.Call(L.ALLREDUCE, count, 7, 0, 2, 0, True), 0)
        want, _ = S.run(algos, plan, [x.copy() for x in ins], [None, None], L.ALLREDUCE, True)
        for r in range(2):
            assert np.array_equal(ts[r].cpu().numpy().view(np.uint32), want[r].view(np.uint32))
    finally:
        for c in comms:
            c.destroy()


def test_c_caller_allreduce(tmp_path):
    """examples/c_allreduce.c (compiled against include/nccl.h) runs a 2-rank grouped AllReduce."""
    import subprocess
    from tests.test_abi import build_c_example
    from msccl_amd import xmlgen
    exe = build_c_example(tmp_path)
    xml = tmp_path / "ap2.xml"
    xml.write_text(xmlgen.allreduce_allpairs(2, 2, "LL"))
    env = dict(os.environ, MSCCL_XML_FILES=str(xml), MSCCL_AMD_TIMEOUT_SEC="20")
    r = subprocess.run([exe, "2", str(8 * 40000)], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("sched", ["allpairs", "pair"])  # pair: the fused exchange (LL)
@pytest.mark.parametrize("proto", ["LL", "Simple"])
def test_hip_graph_capture_and_replay(proto, sched, tmp_path):
    """A grouped AllReduce captured into a hipGraph replays correctly: the launch epoch that
    drives the dependency flags lives on the device (DevComm::epoch), not in the captured
    arguments."""
    import torch
    import msccl_amd as M
    from msccl_amd import xmlgen
    xml = tmp_path / "ap.xml"
    xml.write_text(xmlgen.allreduce_allpairs(2, 2, proto) if sched == "allpairs" else
                   xmlgen.allreduce_pair_oneshot(2, proto))
    os.environ["MSCCL_XML_FILES"] = str(xml)
    n, count = 2, 8 * 5000
    comms = M.Comm.init_all([0] * n)
    try:
        g = torch.Generator().manual_seed(3)
        init = [torch.randint(-4, 5, (count,), generator=g).float() for _ in range(n)]
        bufs = [t.cuda() for t in init]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())

        def step():
            with M.group():
                for c, b in zip(comms, bufs):
                    c.all_reduce(b.data_ptr(), b.data_ptr(), count, M.FLOAT32, M.SUM, s.cuda_stream)

        with torch.cuda.stream(s):
            step()  # eager warm-up launch (epoch 1)
        torch.cuda.synchronize()
        expect = init[0] + init[1]
        for b in bufs:
            assert torch.equal(b.cpu(), expect)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s, capture_error_mode="relaxed"):
            step()
        for k in range(6):
            graph.replay()
            torch.cuda.synchronize()
            expect = expect * 2
            for b in bufs:
                assert torch.equal(b.cpu(), expect), k
        step()  # eager again after replays
        torch.cuda.synchronize()
        expect = expect * 2
        for b in bufs:
            assert torch.equal(b.cpu(), expect)
        for c in comms:
            assert c.async_error() == 0
    finally:
        for c in comms:
            c.destroy()


def test_device_trace_records_every_transfer(tmp_path, monkeypatch):
    """MSCCL_AMD_TRACE=1: every workgroup of the last launch leaves a header, a setup event, a
    begin/end pair per executed transfer and an end event, in time order.  (The interpreter's
    trace: the 2-rank all-pairs is lowered to the fold kernel otherwise, which traces one pass.)"""
    import torch
    import msccl_amd as M
    from msccl_amd import xmlgen
    xml = tmp_path / "ap.xml"
    xml.write_text(xmlgen.allreduce_allpairs(2, 1, "LL"))
    monkeypatch.setenv("MSCCL_XML_FILES", str(xml))
    monkeypatch.setenv("MSCCL_AMD_TRACE", "1")
    monkeypatch.setenv("MSCCL_AMD_LOWER", "0")
    comms = M.Comm.init_all([0, 0])
    try:
        bufs = [torch.ones(4 * 256, device="cuda") for _ in comms]
        for _ in range(3):
            with M.group():
                for c, b in zip(comms, bufs):
                    c.all_reduce(b.data_ptr(), b.data_ptr(), 4 * 256, M.FLOAT32, M.SUM, 0)
        torch.cuda.synchronize()
        algo = M.algo_json(str(xml), 0, 2)
        for c in comms:
            tr = c.trace()
            info = c.info()
            split = info["maxSplit"]
            used = [s for s in range(tr.shape[0]) if tr[s, 0]["type"] == 0xFFFF]
            assert len(used) >= len(algo["tbs"])
            for s in used:
                n = int(tr[s, 0]["step"])
                ev = tr[s, 1:n]
                assert ev[0]["type"] == 1 and ev[-1]["type"] == 5
                assert np.all(np.diff(ev["ts"].astype(np.int64)) >= 0)
                tb = algo["tbs"][s // split]
                assert int((ev["type"] == 3).sum()) == len(tb["transfers"])
                assert int((ev["type"] == 4).sum()) == len(tb["transfers"])
            assert int(tr[used[0], 0]["arg"]) == 3  # epoch of the third launch
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("proto", ["Simple", "LL", "LL128"])
def test_remote_ordering_path(proto, monkeypatch):
    """MSCCL_AMD_FORCE_REMOTE=1 treats every peer as another GPU (system-scope release before a
    Simple tail post, as for xGMI peers): same values, bit-exact."""
    from tests.test_gpu_parity import check
    monkeypatch.setenv("MSCCL_AMD_FORCE_REMOTE", "1")
    check(xmlgen.allreduce_allpairs(4, 2, proto), 4, L.ALLREDUCE, 32 * 5001, 7)
    check(xmlgen.allreduce_ring(4, 2, proto), 4, L.ALLREDUCE, 8 * 7777, 9)


def test_schedules_interleaved_with_multi_workgroup_fold_calls(tmp_path, monkeypatch):
    """Every schedule owns its flag / epoch slots (init.cc: allocSlots).  Fallback calls that run
    the fold kernel with four workgroups (count >= 4 x 512 packs) alternate with a loaded split-1
    all-pairs schedule whose thread blocks wait on each other's flags: a fold launch must never
    advance an epoch another schedule's workgroup has yet to read (before the per-schedule ranges,
    a fold workgroup's epilogue wrote slots 1..3, which other fold workgroups read at their start
    when maxSplit was 1).  Every result bit-exact against the oracle, no wait times out."""
    import torch
    from tests.gpu_harness import CoResident, gen_inputs, to_torch, from_torch
    from oracle import numerics as N
    monkeypatch.setenv("MSCCL_AMD_SPLIT", "1")
    monkeypatch.setenv("MSCCL_AMD_TIMEOUT_SEC", "20")
    n = 2
    xml = xmlgen.allreduce_allpairs(n, 1, "LL", max_bytes=4096)
    dev = torch.device("cuda:0")
    with CoResident(n, [xml], str(tmp_path)) as cr:
        assert cr.comms[0].info()["maxSplit"] == 1
        for it in range(6):
            for count, want_fold in ((4 * 512 * 4, True), (512, False)):
                ins = gen_inputs(n, count, 7, 100 * it + count % 97)
                t = [to_torch(x, dev) for x in ins]
                torch.cuda.synchronize()
                cr.run(L.ALLREDUCE, count, 7, 0, [x.data_ptr() for x in t], [x.data_ptr() for x in t])
                last = cr.comms[0].info()["last"]
                assert (last["small"] == 2 and last["split"] == 4) if want_fold else last["algo"] == 0, last
                want, _ = cr.oracle(L.ALLREDUCE, count, 7, 0, ins, True)
                for r in range(n):
                    got = from_torch(t[r], N.storage(7))
                    assert np.array_equal(got.view(np.uint32), want[r].view(np.uint32)), (it, count, r)

"""NPKit-compatible event log (include/msccl_amd_npkit.h) on the GPU.

Every thread block's buffer must hold, per launch, TIME_SYNC_CPU + TIME_SYNC_GPU and then, for
each transfer of its program, DEP_CHECK_ENTRY/EXIT when it has dependencies and the
primitive's ENTRY/EXIT with the call's bytes (the reference's msccl_interpreter.h:88-201 and
prims_ll.h:455-536 placement).  The dump must be the reference's file set and convert to a
Chrome trace with one B/E pair per recorded interval."""
import os
import time

import numpy as np
import pytest

import msccl_amd as M
from msccl_amd import npkit, xmlgen
from oracle import loader as L
from tests.gpu_harness import CoResident, gen_inputs, to_torch

pytestmark = pytest.mark.gpu
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "20")


def _expected(algo_json, tb, count, ncpl, ts):
    """(event name, size) per launch of thread block `tb` of a one-iteration call: a transfer's
    chunks move as one primitive call (small calls), a reduction per chunk (count-1 here)."""
    per = count // ncpl
    out = [("NPKIT_EVENT_TIME_SYNC_CPU", 0), ("NPKIT_EVENT_TIME_SYNC_GPU", 0)]
    for x in algo_json["tbs"][tb]["transfers"]:
        typ, cnt, ndeps = x[0], x[5], x[7]
        assert typ != 7 or cnt == 1
        if ndeps:
            out += [("NPKIT_EVENT_DEP_CHECK_ENTRY", ndeps), ("NPKIT_EVENT_DEP_CHECK_EXIT", ndeps)]
        name = npkit.TRANSFER_EVENT[typ]
        out += [("NPKIT_EVENT_%s_ENTRY" % name, per * cnt * ts), ("NPKIT_EVENT_%s_EXIT" % name, per * cnt * ts)]
    return out


@pytest.mark.parametrize("proto", ["LL", "Simple"])
def test_npkit_dump_records_every_transfer(tmp_path, monkeypatch, proto):
    import torch
    n, launches, count, dt = 2, 3, 4096, 7
    xml = xmlgen.allreduce_allpairs(n, 1, proto)
    dump = tmp_path / "npkit"
    monkeypatch.setenv("MSCCL_AMD_NPKIT", "1")
    monkeypatch.setenv("MSCCL_AMD_NPKIT_EVENTS", "256")
    monkeypatch.setenv("NPKIT_DUMP_DIR", str(dump))
    t_start = time.time_ns()
    with CoResident(n, [xml], str(tmp_path)) as cr:
        ins = gen_inputs(n, count, dt, 3)
        t = [to_torch(x, torch.device("cuda:0")) for x in ins]
        p = [x.data_ptr() for x in t]
        for _ in range(launches):
            cr.run(L.ALLREDUCE, count, dt, 0, p, p)
        assert all(c.info()["last"]["small"] == 0 for c in cr.comms)  # the log runs the general kernel
        algos = [M.algo_json(cr.paths[0], r, n) for r in range(n)]
    t_end = time.time_ns()
    files = set(os.listdir(dump))
    for r in range(n):
        for b in range(npkit.GPU_BUFFERS):
            assert "gpu_events_rank_%d_buf_%d" % (r, b) in files
        for c in range(npkit.CPU_BUFFERS):
            assert os.path.getsize(dump / ("cpu_events_rank_%d_channel_%d" % (r, c))) == 0
        assert (dump / ("cpu_clock_period_den_rank_%d" % r)).read_text() == "1000000000"
        khz = float((dump / ("gpu_clock_rate_rank_%d" % r)).read_text())
        assert khz > 0
        a = algos[r]
        for tb in range(len(a["tbs"])):
            ev = npkit.read_buffer(str(dump), r, tb)
            want = _expected(a, tb, count, a["nchunksperloop"], 4) * launches
            got = [(npkit.NAMES[e["id"]], e["size"]) for e in ev]
            assert got == want, "rank %d tb %d" % (r, tb)
            # host time of each launch start: inside the test's window (calibrated clock)
            for e in ev:
                if e["id"] == npkit.EVENTS["NPKIT_EVENT_TIME_SYNC_CPU"]:
                    assert t_start - 1_000_000 <= e["timestamp"] <= t_end + 1_000_000
            # GPU clock non-decreasing within the buffer
            gts = [e["timestamp"] for e in ev if e["id"] != npkit.EVENTS["NPKIT_EVENT_TIME_SYNC_CPU"]]
            assert all(x <= y for x, y in zip(gts, gts[1:]))
        for tb in range(len(a["tbs"]), npkit.GPU_BUFFERS):
            assert os.path.getsize(dump / ("gpu_events_rank_%d_buf_%d" % (r, tb))) == 0
    tr = npkit.to_trace(str(dump))["traceEvents"]
    b = [e for e in tr if e["ph"] == "B"]
    e = [e for e in tr if e["ph"] == "E"]
    assert len(b) == len(e) > 0
    assert all(x["cat"] == "GPU" for x in b)
    assert {x["name"] for x in b} >= {"SEND", "RECV_REDUCE_COPY"} or {x["name"] for x in b} >= {"SEND", "RECV"}


def test_npkit_buffer_cap_and_explicit_dump(tmp_path, monkeypatch):
    """Events past MSCCL_AMD_NPKIT_EVENTS are dropped, not written out of bounds; the buffer
    keeps its first events across launches; mscclAmdNpkitDump writes on demand."""
    import torch
    n, count, dt = 2, 1024, 7
    xml = xmlgen.allreduce_pair_oneshot(1, "LL")
    monkeypatch.setenv("MSCCL_AMD_NPKIT", "1")
    monkeypatch.setenv("MSCCL_AMD_NPKIT_EVENTS", "16")
    monkeypatch.setenv("NPKIT_DUMP_DIR", str(tmp_path / "at_destroy"))
    with CoResident(n, [xml], str(tmp_path)) as cr:
        t = [to_torch(x, torch.device("cuda:0")) for x in gen_inputs(n, count, dt, 1)]
        p = [x.data_ptr() for x in t]
        for _ in range(10):  # 6 events per launch (sync x2, s, rrc): 60 > 16
            cr.run(L.ALLREDUCE, count, dt, 0, p, p)
        cr.comms[0].npkit_dump(str(tmp_path / "explicit"))
    ev = npkit.read_buffer(str(tmp_path / "explicit"), 0, 0)
    assert len(ev) == 16
    names = [npkit.NAMES[e["id"]] for e in ev]
    assert names[:6] == ["NPKIT_EVENT_TIME_SYNC_CPU", "NPKIT_EVENT_TIME_SYNC_GPU", "NPKIT_EVENT_SEND_ENTRY",
                         "NPKIT_EVENT_SEND_EXIT", "NPKIT_EVENT_RECV_REDUCE_COPY_ENTRY",
                         "NPKIT_EVENT_RECV_REDUCE_COPY_EXIT"]
    assert names[6:12] == names[:6]
    assert len(npkit.read_buffer(str(tmp_path / "at_destroy"), 1, 0)) == 16


def test_npkit_off_by_default(tmp_path):
    xml = xmlgen.allreduce_pair_oneshot(1, "LL")
    with CoResident(2, [xml], str(tmp_path)) as cr:
        with pytest.raises(M.NcclError):
            cr.comms[0].npkit_dump(str(tmp_path / "x"))


def test_npkit_and_trace_cover_the_fold_kernel(tmp_path, monkeypatch):
    """A fallback call that runs the flat fold kernel (no schedule loaded, the flat tree) still
    logs: per launch TIME_SYNC_CPU / TIME_SYNC_GPU and its one pass as RECV_REDUCE_COPY_SEND with
    the call's bytes in thread block 0's buffer; MSCCL_AMD_TRACE=1 records the workgroup's setup,
    primitive begin / end and end events."""
    import torch
    n, launches, count, dt = 2, 3, 1000, 7
    monkeypatch.setenv("NCCL_ALGO", "Ring,Tree")
    monkeypatch.setenv("MSCCL_AMD_NPKIT", "1")
    monkeypatch.setenv("MSCCL_AMD_NPKIT_EVENTS", "64")
    monkeypatch.setenv("MSCCL_AMD_TRACE", "1")
    with CoResident(n, [], str(tmp_path)) as cr:
        t = [to_torch(x, torch.device("cuda:0")) for x in gen_inputs(n, count, dt, 5)]
        p = [x.data_ptr() for x in t]
        for _ in range(launches):
            cr.run(L.ALLREDUCE, count, dt, 0, p, p)
        last = cr.comms[0].info()["last"]
        assert last["ringColl"] == 5 and last["small"] == 2, last
        tr = cr.comms[0].trace()
        cr.comms[0].npkit_dump(str(tmp_path / "fold"))
    hdr = tr[0, 0]
    assert hdr["type"] == 0xFFFF and hdr["step"] == 5
    assert [M.TRACE_TYPES.get(int(e["type"])) for e in tr[0, 1:5]] == [M.TRACE_TYPES[k] for k in (1, 3, 4, 5)]
    ev = npkit.read_buffer(str(tmp_path / "fold"), 0, 0)
    got = [(npkit.NAMES[e["id"]], e["size"]) for e in ev]
    want = [("NPKIT_EVENT_TIME_SYNC_CPU", 0), ("NPKIT_EVENT_TIME_SYNC_GPU", 0),
            ("NPKIT_EVENT_RECV_REDUCE_COPY_SEND_ENTRY", count * 4),
            ("NPKIT_EVENT_RECV_REDUCE_COPY_SEND_EXIT", count * 4)] * launches
    assert got == want

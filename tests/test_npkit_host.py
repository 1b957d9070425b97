"""NPKit host side, no GPU: the event table mirrors include/msccl_amd_npkit.h; the converter's
arithmetic on hand-worked dumps (the reference generator's rules, tools/npkit_trace_generator.py:
72-127 GPU events, 129-189 CPU fibers); and its output on a real dump of the product
(tests/golden/npkit/dump.tar.gz).  Running the reference generator itself here was refused, so
equality with its output is unpinned."""
import json
import os
import re
import tarfile

import pytest

from msccl_amd import npkit

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "npkit")


def test_event_table_matches_header():
    text = open(os.path.join(ROOT, "include", "msccl_amd_npkit.h")).read()
    hdr = {m.group(1): int(m.group(2), 0) for m in re.finditer(r"#define (NPKIT_EVENT_\w+) (0x[0-9A-Fa-f]+)", text)}
    assert hdr == npkit.EVENTS


def test_event_parse_layout():
    raw = bytes([0x1B]) + (1234).to_bytes(4, "little") + (77).to_bytes(3, "little") + (99).to_bytes(8, "little")
    assert npkit.parse_events(raw) == [{"id": 0x1B, "size": 1234, "rsvd": 77, "timestamp": 99}]


def test_converter_on_product_dump(tmp_path):
    """2 ranks x 2 thread blocks x 4 launches of a 2-rank all-pairs LL AllReduce (16384 fp32):
    every interval is a B/E pair on its (rank, buffer) track, in time order, with the call's bytes;
    every launch's intervals sit after its TIME_SYNC point on the host timeline."""
    with tarfile.open(os.path.join(GOLD, "dump.tar.gz")) as t:
        t.extractall(tmp_path, filter="data")
    tr = npkit.to_trace(str(tmp_path))
    ev = tr["traceEvents"]
    assert tr["displayTimeUnit"] == "ns" and ev == sorted(ev, key=lambda e: e["ts"])
    tracks = {}
    for e in ev:
        tracks.setdefault((e["pid"], e["tid"]), []).append(e)
    assert set(tracks) == {(0, 1), (0, 2), (1, 1), (1, 2)}
    for (rank, tid), es in tracks.items():
        raw = [x for x in npkit.read_buffer(str(tmp_path), rank, tid - 1)
               if npkit.NAMES[x["id"]] not in ("NPKIT_EVENT_TIME_SYNC_CPU", "NPKIT_EVENT_TIME_SYNC_GPU")]
        assert len(es) == len(raw) and len(es) % 2 == 0
        for b, e in zip(es[0::2], es[1::2]):
            assert b["ph"] == "B" and e["ph"] == "E" and b["ts"] <= e["ts"]
            assert b["args"]["size_0"] == e["args"]["size"] > 0
            assert b["args"]["buf_idx"] == tid - 1 and b["args"]["rank"] == rank
        names = [b["name"] for b in es[0::2]]
        per_launch = len(names) // 4
        assert names == names[:per_launch] * 4  # the same program every launch
        # the sequence numbers count each event type on its own
        for nm in set(names):
            assert [b["args"]["seq"] for b in es[0::2] if b["name"] == nm] == list(range(names.count(nm)))


def test_cli_writes_trace(tmp_path):
    d = tmp_path / "dump"
    d.mkdir()
    ev = b"".join(
        bytes([t]) + s.to_bytes(4, "little") + b"\0\0\0" + ts.to_bytes(8, "little")
        for t, s, ts in [(0x2C, 0, 1_000_000), (0x2B, 0, 500), (0x1, 64, 600), (0x2, 64, 700)])
    (d / "gpu_events_rank_0_buf_0").write_bytes(ev)
    (d / "cpu_events_rank_0_channel_0").write_bytes(b"")
    (d / "cpu_clock_period_num_rank_0").write_text("1")
    (d / "cpu_clock_period_den_rank_0").write_text("1000000000")
    (d / "gpu_clock_rate_rank_0").write_text("100000")
    npkit.main(["--input_dir", str(d), "--output_dir", str(tmp_path / "out")])
    tr = json.load(open(tmp_path / "out" / "npkit_event_trace.json"))
    assert tr["displayTimeUnit"] == "ns"
    b, e = tr["traceEvents"]
    # cpu base 1e6 ns = 1000 us; gpu 100 ticks/us: entry 1 us after the sync, exit 1 us later
    assert b["ph"] == "B" and b["name"] == "SEND" and b["ts"] == pytest.approx(1001.0)
    assert e["ph"] == "E" and e["ts"] == pytest.approx(1002.0) and e["args"]["bw (GB/s)"] == pytest.approx(0.064)

"""bench.py's schedule tiers: contiguous cover of the sweep, at most MSCCL_MAX_NUM_ALGOS (4) XMLs,
every XML valid on every rank (product loader), and every default sweep size divisible by its
tier's nchunksperloop, so no sweep point is silently skipped (CPU only)."""
import sys

import pytest

import msccl_amd as M


@pytest.fixture(scope="module")
def bench():
    argv = sys.argv
    sys.argv = ["bench.py"]
    try:
        import bench as B
    finally:
        sys.argv = argv
    return B


@pytest.mark.parametrize("n,inst,ts", [(2, 16, 4), (4, 8, 4), (8, 4, 2)])
def test_default_tiers_cover_the_sweep(bench, tmp_path, n, inst, ts):
    tiers = bench.make_xmls(n, "LL", inst, str(tmp_path))
    assert 1 <= len(tiers) <= 4
    assert tiers[0][0] == 0
    for a, b in zip(tiers, tiers[1:]):
        assert a[1] == b[0]
    assert tiers[-1][1] > max(bench.SIZES)
    for lo, hi, i, path, kind in tiers:
        for r in range(n):
            j = M.algo_json(path, r, n)
            assert j["valid"] == 1 and j["minBytes"] == lo and j["maxBytes"] == hi
    for nbytes in bench.SIZES:
        t = bench.tier_of(tiers, nbytes)
        ncpl = t[2] * (n * n if t[4] == "a" else 1)
        assert (nbytes // ts) % ncpl == 0, (nbytes, t)


def test_tier_spec_with_kinds(bench, tmp_path):
    tiers = bench.make_xmls(2, "LL", 16, str(tmp_path), "0:4096:1:o,4096:65536:2:O,65536:1073741825:4")
    assert [t[4] for t in tiers] == ["o", "O", "a"]
    assert [t[2] for t in tiers] == [1, 2, 4]


def test_workload_label_names_the_schedule_that_ran(bench):
    """config.workload names the headline size's schedule: "all-pairs" only on an all-pairs XML,
    and the pair one-shot says it is not one."""
    a = bench.workload_desc(False, 2, "LL", "fp32", kind="a")
    assert a.startswith("C2: ") and "msccl-tools two-phase all-pairs XML" in a
    p = bench.workload_desc(False, 2, "LL", "fp32", kind="p")
    assert "pair one-shot" in p and "not all-pairs" in p
    assert "all-pairs" not in p.replace("not all-pairs", "")
    assert "C3 shape: " in bench.workload_desc(False, 8, "LL", "fp16", kind="a")
    assert "over xGMI" in bench.workload_desc(True, 8, "LL", "fp16", kind="a")
    assert "rehearsal" in bench.workload_desc(True, 8, "LL", "fp16", one_gpu=True, kind="O")
    assert bench.parse(["--no-tuning"]).no_tuning


def test_secondary_lines_and_tuning_grid(bench):
    """Beside a 2-rank headline (the all-pairs XML) the secondary line is the pair one-shot; at more
    ranks the two-phase all-pairs x4 (and at N=1 RCCL's 8n-32tb file when installed).  The tuning
    grid of bench.py --gpus N is the one DESIGN.md §6 / §10.4 names."""
    two = bench.secondary_schedules(False, 2, 32 << 20)
    assert two[0][0] == "pair_oneshot" and 'name="sec_pair"' in two[0][1], two[0][1][:200]
    eight = bench.secondary_schedules(True, 8, 32 << 20)
    assert [s[0] for s in eight] == ["allpairs_two_phase"]
    assert bench.TUNE_SIZES == (64 << 10, 128 << 10, 256 << 10, 512 << 10, 1 << 20)
    assert bench.TUNE_LOWER_CAPS == (128 << 10, 256 << 10, 512 << 10)
    assert bench.TUNE_BUFFSIZES == (256 << 10, 4 << 20)


def test_fused_pair_exchange_bytes(bench, tmp_path):
    """The roofline's algorithmic bytes: the pair exchange moves 7 S HBM bytes per rank unfused
    (s: S + 2S of LL lines, rrc: 2S + S + S) and 6 S when its s + rrc run fused (the source is
    read once; comm info "algoFuse" names the fused thread blocks)."""
    p = tmp_path / "pair.xml"
    p.write_text(bench.xmlgen.allreduce_pair_oneshot(16, "LL"))
    algo = M.algo_json(str(p), 0, 2)
    size_per, ts = 1 << 16, 4
    S = 16 * size_per * ts
    assert bench.schedule_bytes(algo, size_per, ts, 0)[0] == 7 * S
    assert bench.schedule_bytes(algo, size_per, ts, 0, fused=set(range(16)))[0] == 6 * S
    assert bench.schedule_bytes(algo, size_per, ts, 0, payload_only=True, fused=set(range(16)))[0] == 4 * S
    assert bench.schedule_bytes(algo, size_per, ts, 2, fused=set(range(16)))[0] == 5 * S  # Simple: not fused

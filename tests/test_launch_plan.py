"""What a communicator launches, with init's decisions, by placement (plan.cc: planCall through
mscclAmdLaunchPlanJson; no GPU): the one-hop lowering limit from the link model for ranks on
different GPUs against the measured co-resident limit, the local Simple FIFO, the
trace / NPKit rule that keeps a schedule interpreted."""
import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from oracle import loader as L


def _files(tmp_path, xmls):
    paths = []
    for i, x in enumerate(xmls):
        p = tmp_path / ("s%d.xml" % i)
        p.write_text(x)
        paths.append(str(p))
    return ":".join(paths)


def test_link_model_defaults():
    """The remote limit is the model's crossover (dF + L) B / (f (1 - 2/n)) floored to a power of
    two and capped at 256 KiB; co-resident ranks keep the measured 4 KiB / 128 KiB; two ranks keep
    4 KiB (the pair exchange is already one hop with the fold's link bytes)."""
    b_us = 76.8e3                     # one xGMI link, one way, bytes per microsecond
    for n in (3, 4, 8, 16):
        x = (5.0 + 2.0) * b_us / (2.0 * (1 - 2.0 / n))
        p = 4096
        while p * 2 <= x and p * 2 <= 256 << 10:
            p *= 2
        assert p == 256 << 10        # every n >= 3 reaches the cap with these parameters
    xml = xmlgen.allreduce_allpairs(8, 1, "LL")
    import tempfile
    import os
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "a.xml")
        open(path, "w").write(xml)
        for one_gpu, want in ((True, 128 << 10), (False, 256 << 10)):
            got = M.launch_plan_json(path, 0, 8, one_gpu, L.ALLREDUCE, 1024, 7, 0, True)
            assert got["lowerMaxBytes"] == want, got
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "p.xml")
        open(path, "w").write(xmlgen.allreduce_pair_oneshot(16, "LL"))
        for one_gpu in (True, False):
            assert M.launch_plan_json(path, 0, 2, one_gpu, L.ALLREDUCE, 1024, 7, 0, True)["lowerMaxBytes"] == 4096


@pytest.mark.parametrize("nbytes,co,remote", [
    (128, "fold", "fold"), (64 << 10, "fold", "fold"), (128 << 10, "fold", "fold"),
    (256 << 10, "twophase", "fold"), (512 << 10, "twophase", "twophase"),
    (32 << 20, "twophase", "twophase")])
def test_c3_tiers_by_placement(tmp_path, nbytes, co, remote):
    """bench.py's 8-rank tiers (C3, fp16): up to 128 KiB both placements run the fold; at 256 KiB
    only ranks on different GPUs do (the link model); above, the two-phase all-pairs tiers run
    their two-phase form (lower.h: FoldLowering::twoPhase), on either placement."""
    import bench
    tiers = bench.make_xmls(8, "LL", 8, str(tmp_path))
    files = ":".join(t[3] for t in tiers)
    for one_gpu, want in ((True, co), (False, remote)):
        got = M.launch_plan_json(files, 3, 8, one_gpu, L.ALLREDUCE, nbytes // 2, 6, 0, True)
        assert got["kernel"] == want, (one_gpu, got)
        assert got["lowered"] == 1
        assert got["remote"] == (0 if one_gpu else 1)
    import os
    os.environ["MSCCL_AMD_LOWER_LARGE"] = "0"
    try:
        for one_gpu, want in ((True, co), (False, remote)):
            got = M.launch_plan_json(files, 3, 8, one_gpu, L.ALLREDUCE, nbytes // 2, 6, 0, True)
            assert got["kernel"] == (want if want == "fold" else "interpreter"), (one_gpu, got)
    finally:
        del os.environ["MSCCL_AMD_LOWER_LARGE"]


def test_lower_limit_knob_overrides_both(tmp_path, monkeypatch):
    files = _files(tmp_path, [xmlgen.allreduce_allpairs(8, 1, "LL")])
    monkeypatch.setenv("MSCCL_AMD_LOWER_MAX_BYTES", "8192")
    for one_gpu in (True, False):
        got = M.launch_plan_json(files, 0, 8, one_gpu, L.ALLREDUCE, 16384 // 4, 7, 0, True)
        assert got["lowerMaxBytes"] == 8192 and got["kernel"] == "twophase", got
    monkeypatch.setenv("MSCCL_AMD_LOWER_LARGE", "0")
    for one_gpu in (True, False):
        got = M.launch_plan_json(files, 0, 8, one_gpu, L.ALLREDUCE, 16384 // 4, 7, 0, True)
        assert got["lowerMaxBytes"] == 8192 and got["kernel"] == "interpreter", got


@pytest.mark.parametrize("env", ["MSCCL_AMD_TRACE=1", "MSCCL_AMD_NPKIT=1", "MSCCL_AMD_LOWER=0"])
def test_traced_schedule_runs_as_written(tmp_path, monkeypatch, env):
    """A full trace or NPKit records the schedule's own primitives: no lowering."""
    files = _files(tmp_path, [xmlgen.allreduce_allpairs(8, 1, "LL")])
    assert M.launch_plan_json(files, 0, 8, True, L.ALLREDUCE, 1024, 7, 0, True)["kernel"] == "fold"
    k, v = env.split("=")
    monkeypatch.setenv(k, v)
    got = M.launch_plan_json(files, 0, 8, True, L.ALLREDUCE, 1024, 7, 0, True)
    assert got["kernel"] == "interpreter" and got["classes"] == [0], got


def test_light_trace_keeps_lowering(tmp_path, monkeypatch):
    files = _files(tmp_path, [xmlgen.allreduce_allpairs(8, 1, "LL")])
    monkeypatch.setenv("MSCCL_AMD_TRACE", "2")
    assert M.launch_plan_json(files, 0, 8, True, L.ALLREDUCE, 1024, 7, 0, True)["kernel"] == "fold"


def test_local_simple_fifo_by_placement(tmp_path, monkeypatch):
    """256 KiB Simple FIFO only when every rank shares one GPU, NCCL_BUFFSIZE is unset and no
    Simple schedule sends more than two chunks before it receives (init.cc: applySplits)."""
    ring = _files(tmp_path, [xmlgen.allreduce_ring(8, 4, "Simple", True)])
    assert M.launch_plan_json(ring, 0, 8, True, L.ALLREDUCE, 1 << 20, 9, 0, True)["simpleBuffBytes"] == 256 << 10
    assert M.launch_plan_json(ring, 0, 8, False, L.ALLREDUCE, 1 << 20, 9, 0, True)["simpleBuffBytes"] == 4 << 20
    monkeypatch.setenv("NCCL_BUFFSIZE", str(1 << 20))
    assert M.launch_plan_json(ring, 0, 8, True, L.ALLREDUCE, 1 << 20, 9, 0, True)["simpleBuffBytes"] == 1 << 20


def test_fallback_and_ll128_remote(tmp_path):
    """No schedule matches: the flat fold (LL range) or the ring; an LL128 schedule runs as LL
    across GPUs (the line-tear gate) and as LL128 on one GPU."""
    files = _files(tmp_path, [xmlgen.allreduce_allpairs(4, 1, "LL128")])
    assert M.launch_plan_json(files, 0, 4, True, L.ALLREDUCE, 1 << 14, 7, 0, True)["proto"] == 1
    assert M.launch_plan_json(files, 0, 4, False, L.ALLREDUCE, 1 << 14, 7, 0, True)["proto"] == 0
    got = M.launch_plan_json(files, 0, 4, False, L.ALLREDUCE, 1001, 7, 0, True)
    assert got["kernel"] == "fold" and got["algo"] == -1, got
    got = M.launch_plan_json(files, 0, 4, False, L.ALLREDUCE, (8 << 20) + 1, 7, 0, True)
    assert got["kernel"] == "ring", got


def test_pair_form_schedule_keeps_the_pair_kernel(tmp_path, monkeypatch):
    """A schedule in pair form (every thread block one fused s + rrc, transport.cc: pairFormOf) is
    not lowered by default on either placement: the pair kernel's fixed cost is the fold's or less
    (init.cc: applySplits).  An explicit MSCCL_AMD_LOWER_MAX_BYTES, MSCCL_AMD_PAIR_KERNEL=0 or
    MSCCL_AMD_FUSE=0 brings the fold back; the two-phase all-pairs (not pair form) stays lowered."""
    files = _files(tmp_path, [xmlgen.allreduce_pair_oneshot(1, "LL")])
    for one_gpu in (True, False):
        got = M.launch_plan_json(files, 0, 2, one_gpu, L.ALLREDUCE, 32, 7, 0, True)
        assert got["kernel"] == "pair" and got["classes"] == [0], got
    for env in (("MSCCL_AMD_LOWER_MAX_BYTES", "4096"), ("MSCCL_AMD_PAIR_KERNEL", "0"), ("MSCCL_AMD_FUSE", "0")):
        monkeypatch.setenv(*env)
        got = M.launch_plan_json(files, 0, 2, True, L.ALLREDUCE, 32, 7, 0, True)
        assert got["kernel"] == "fold" and got["classes"] == [1], (env, got)
        monkeypatch.delenv(env[0])
    files = _files(tmp_path, [xmlgen.allreduce_allpairs(2, 4, "LL")])
    got = M.launch_plan_json(files, 0, 2, True, L.ALLREDUCE, 32, 7, 0, True)
    assert got["kernel"] == "fold", got


@pytest.mark.parametrize("nbytes", [128, 8192, 1 << 20, 32 << 20])
def test_c2_tiers_launch_the_pair_kernel(tmp_path, nbytes):
    """The pair one-shot tiers (bench.PAIR_TIERS): every size from 128 B to 32 MiB is a pair-form
    call that runs the pair kernel in one pass, on one GPU and across GPUs."""
    import bench
    tiers = bench.make_xmls(2, "LL", 16, str(tmp_path), bench.PAIR_TIERS)
    files = ":".join(t[3] for t in tiers)
    for one_gpu in (True, False):
        got = M.launch_plan_json(files, 0, 2, one_gpu, L.ALLREDUCE, nbytes // 4, 7, 0, True)
        assert got["kernel"] == "pair" and got["pairForm"] == 1, (one_gpu, got)


@pytest.mark.parametrize("nbytes,kernel", [(128, "fold"), (4080, "fold"), (8192, "pair"), (1 << 20, "pair"),
                                           (32 << 20, "pair")])
def test_c2_default_tiers_run_the_allpairs_xml_lowered(tmp_path, nbytes, kernel):
    """bench.py's C2 tiers (the msccl-tools two-phase all-pairs XML): lowered at every size, the
    one-hop fold up to 4 KiB and the pair exchange on the flat connections above, either placement."""
    import bench
    tiers = bench.make_xmls(2, "LL", 16, str(tmp_path))
    assert [t[4] for t in tiers] == ["a", "a"]
    files = ":".join(t[3] for t in tiers)
    for one_gpu in (True, False):
        got = M.launch_plan_json(files, 0, 2, one_gpu, L.ALLREDUCE, nbytes // 4, 7, 0, True)
        assert got["kernel"] == kernel and got["lowered"] == 1 and got["pairForm"] == 0, (one_gpu, got)


def test_pair_kernel_knob_and_non_pair_schedules(tmp_path, monkeypatch):
    files = _files(tmp_path, [xmlgen.allreduce_pair_oneshot(16, "LL")])
    monkeypatch.setenv("MSCCL_AMD_PAIR_KERNEL", "0")
    got = M.launch_plan_json(files, 0, 2, True, L.ALLREDUCE, 1 << 18, 7, 0, True)
    # lowered instead (the pair kernel off the table leaves the schedule to the lowering): the
    # lowered pair runs the pair kernel on the flat connections on both ends whatever the
    # rank-local knob says
    assert got["kernel"] == "pair" and got["lowered"] == 1 and got["pairForm"] == 1, got
    monkeypatch.setenv("MSCCL_AMD_LOWER_LARGE", "0")
    got = M.launch_plan_json(files, 0, 2, True, L.ALLREDUCE, 1 << 18, 7, 0, True)
    assert got["kernel"] == "interpreter" and got["pairForm"] == 1, got
    monkeypatch.delenv("MSCCL_AMD_LOWER_LARGE")
    monkeypatch.delenv("MSCCL_AMD_PAIR_KERNEL")
    files = _files(tmp_path, [xmlgen.allreduce_allpairs(2, 16, "LL")])
    got = M.launch_plan_json(files, 0, 2, True, L.ALLREDUCE, 1 << 20, 7, 0, True)
    # the two-phase all-pairs of 2 ranks: its large calls run lowered as the pair exchange
    assert got["kernel"] == "pair" and got["lowered"] == 1 and got["pairForm"] == 0, got
    monkeypatch.setenv("MSCCL_AMD_LOWER_LARGE", "0")
    got = M.launch_plan_json(files, 0, 2, True, L.ALLREDUCE, 1 << 20, 7, 0, True)
    assert got["kernel"] == "interpreter" and got["pairForm"] == 0, got
    monkeypatch.delenv("MSCCL_AMD_LOWER_LARGE")
    # a call of more than 64 iterations stays on the interpreter (the one-pass merge caps at 64)
    files = _files(tmp_path, [xmlgen.allreduce_pair_oneshot(1, "LL")])
    got = M.launch_plan_json(files, 0, 2, True, L.ALLREDUCE, 1 << 24, 7, 0, True)
    assert got["kernel"] == "interpreter" and got["pairForm"] == 1, got
    assert got["kernelExact"] == 1, got


def test_pair_answer_flagged_approximate_off_the_default_fifo(tmp_path, monkeypatch):
    """for a multi-iteration pair-form call the one-pass bound rests on the default LL
    FIFO and split; under NCCL_LL_BUFFSIZE or MSCCL_AMD_SPLIT the answer says it is approximate."""
    files = _files(tmp_path, [xmlgen.allreduce_pair_oneshot(1, "LL")])
    got = M.launch_plan_json(files, 0, 2, True, L.ALLREDUCE, 1 << 18, 7, 0, True)
    assert got["kernelExact"] == 1, got
    for env in (("NCCL_LL_BUFFSIZE", str(1 << 18)), ("MSCCL_AMD_SPLIT", "2")):
        monkeypatch.setenv(*env)
        got = M.launch_plan_json(files, 0, 2, True, L.ALLREDUCE, 1 << 18, 7, 0, True)
        assert got["kernelExact"] == 0, (env, got)
        small = M.launch_plan_json(files, 0, 2, True, L.ALLREDUCE, 32, 7, 0, True)
        assert small["kernelExact"] == 1, (env, small)   # one iteration: exact
        monkeypatch.delenv(env[0])

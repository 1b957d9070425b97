"""bench.py's launcher (CPU only): `bench.py --gpus N` runs N ranks, one per GPU, started by
itself when torch.distributed.run did not start it (the reference's harness: `mpirun -np 8 ...
all_reduce_perf -g 1`, README.md:57), refuses when fewer GPUs are visible, and keeps the one-GPU
rehearsal behind MSCCL_AMD_BENCH_ONE_GPU=1."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    argv = sys.argv
    sys.argv = ["bench.py"]
    try:
        import bench as B
    finally:
        sys.argv = argv
    return B


def test_default_is_one_process_c2(bench):
    assert bench.launch_plan(None, {}, 1) == ("local", 1)
    assert bench.launch_plan(1, {}, 8) == ("local", 1)
    assert bench.launch_plan(None, {}, 0)[0] == "local"   # the CPU-only box: N=1 needs no count


@pytest.mark.parametrize("n", [2, 4, 8])
def test_spawns_n_ranks_when_enough_gpus(bench, n):
    assert bench.launch_plan(n, {}, 8) == ("spawn", n)


@pytest.mark.parametrize("n,devs", [(2, 1), (8, 4), (8, 1), (2, 0)])
def test_refuses_fewer_gpus_than_ranks(bench, n, devs):
    mode, why = bench.launch_plan(n, {}, devs)
    assert mode == "refuse" and "MSCCL_AMD_BENCH_ONE_GPU" in why


def test_one_gpu_knob_rehearses(bench):
    env = {"MSCCL_AMD_BENCH_ONE_GPU": "1"}
    assert bench.launch_plan(2, env, 1) == ("spawn", 2)
    assert bench.launch_plan(2, dict(env, WORLD_SIZE="2"), 1) == ("rank", 2)


def test_under_torchrun_each_process_is_a_rank(bench):
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}, 8) == ("rank", 8)
    assert bench.launch_plan(None, {"WORLD_SIZE": "8"}, 8) == ("rank", 8)
    assert bench.launch_plan(4, {"WORLD_SIZE": "8"}, 8)[0] == "refuse"     # --gpus disagrees
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}, 2)[0] == "refuse"     # too few devices
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}, 1) == ("local", 1)


def test_cli_refuses_without_gpus():
    """No GPU here: `bench.py --gpus 2` must exit non-zero with the reason, before any GPU work."""
    env = dict(os.environ)
    env.pop("MSCCL_AMD_BENCH_ONE_GPU", None)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2
    assert "needs 2 GPUs" in r.stderr
    assert r.stdout == ""


def test_spawn_command(bench, monkeypatch):
    calls = []
    monkeypatch.setattr(subprocess, "call", lambda cmd: calls.append(cmd) or 0)
    assert bench.spawn_ranks(4, ["--gpus", "4", "--steps", "3"]) == 0
    cmd = calls[0]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-3:] == ["4", "--steps", "3"] and cmd[-4] == "--gpus"

"""CPU tests of bench.py's launch logic: `--gpus N` without a torchrun
environment starts N ranks itself, and a torchrun world that disagrees with
--gpus is refused before anything touches a GPU."""
import argparse
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def _args(gpus, cpu_threads=0):
    return argparse.Namespace(gpus=gpus, cpu_threads=cpu_threads)


def test_one_gpu_runs_in_process():
    assert bench.resolve_launch(_args(1), env={}) == ("rank", 1)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_n_gpus_without_torchrun_spawns_n_ranks(n):
    assert bench.resolve_launch(_args(n), env={}) == ("spawn", n)


@pytest.mark.parametrize("n", [1, 2, 8])
def test_torchrun_world_matching_gpus_is_a_rank(n):
    assert bench.resolve_launch(_args(n), env={"WORLD_SIZE": str(n)}) == ("rank", n)


@pytest.mark.parametrize("gpus,world", [(2, 1), (8, 1), (1, 2), (8, 4)])
def test_world_mismatch_is_refused(gpus, world):
    with pytest.raises(SystemExit, match="WORLD_SIZE"):
        bench.resolve_launch(_args(gpus), env={"WORLD_SIZE": str(world)})


def test_zero_gpus_is_refused():
    with pytest.raises(SystemExit):
        bench.resolve_launch(_args(0), env={})


def test_guard_fires_from_the_command_line():
    """The real entry point: a 1-rank torchrun world asked for 8 GPUs exits
    non-zero with the guard's message, before any GPU work."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "8"],
                       capture_output=True, text=True, timeout=180, env=env, cwd=ROOT)
    assert r.returncode != 0
    assert "--gpus 8 but WORLD_SIZE=1" in r.stderr
    assert not any(l.startswith("{") for l in r.stdout.splitlines())


def test_cpu_baseline_threads(monkeypatch):
    visible = len(os.sched_getaffinity(0))
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    assert bench.cpu_threads(_args(1))[0] == visible
    if visible > 1:
        monkeypatch.setenv("OMP_NUM_THREADS", "1")
        th, vis, why = bench.cpu_threads(_args(1))
        assert (th, vis) == (1, visible) and "OMP_NUM_THREADS" in why
    assert bench.cpu_threads(_args(1, cpu_threads=3))[0] == 3

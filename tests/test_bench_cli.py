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


@pytest.mark.parametrize("batch,want", [(64 << 20, 16), (1 << 30, 1), (1543503872, 1),
                                        (268435456, 4), (134217728, 8), (9000 << 20, 1),
                                        ((1 << 30) - 1, 2)])
def test_rotation_covers_the_infinity_cache(batch, want):
    """Strided batches rotate over ceil(1 GiB / batch) distinct batches, so
    the footprint is >= 4x the 256 MiB Infinity Cache (C3 64 B: 16 x 67 MB;
    C2's 1.54 GB batch: 1)."""
    a = bench.parse([])
    assert bench.rotation(batch, a) == want
    assert bench.rotation(batch, bench.parse(["--batches", "4"])) == 4


def test_default_line_carries_the_secondary_legs():
    a = bench.parse([])
    assert not a.no_extra and a.c3_packets == 1 << 20 and a.c4_packets == 1 << 24
    assert bench.C3_SIZES == (64, 256, 576, 1472, 9000)

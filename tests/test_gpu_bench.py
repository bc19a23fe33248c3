"""bench.py contract on the GPU box: the 1-GPU JSON line, and the N-rank path
rehearsed as 2 ranks sharing cuda:0 over gloo (the 8-GPU RCCL run is the
driver's)."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
        "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
        "roofline", "cpu_baseline"}


def _last_json(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_one_gpu_line(gpu):
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "5", "--warmup", "1",
                        "--packets", "65536", "--cpu-seconds", "0.5"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert KEYS <= set(line)
    assert line["n_gpus"] == 1 and line["steps"] == 5 and line["value"] > 0
    assert line["roofline"]["bound"] == "hbm" and 0 < line["roofline"]["frac"] < 1.5
    assert line["cpu_baseline"]["kind"] == "port" and line["cpu_baseline"]["cores"] >= 1
    assert line["parity"]["mismatches"] == 0


def test_bench_two_ranks_rehearsal(gpu):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, WC_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", str(port), str(ROOT / "bench.py"), "--gpus", "2",
                        "--steps", "5", "--warmup", "1", "--packets", "65536"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["cpu_baseline"] is None
    assert line["parity"] == {"checked_packets": 2 * 65536, "mismatches": 0}
    assert line["results_allgather"]["ranks_mismatched"] == 0
    assert line["results_allgather"]["bytes_per_rank"] == 2 * 65536


@pytest.mark.parametrize("args", [["--config", "c4", "--packets", "200000"],
                                  ["--config", "c4", "--packets", "200000", "--kind", "payload",
                                   "--headers"],
                                  ["--config", "slots", "--packets", "65536", "--kind", "payload",
                                   "--headers"],
                                  ["--config", "c2", "--packets", "65536", "--kind", "payload"]])
def test_bench_other_configs(gpu, args):
    """The secondary bench lines (C4, payload_cksum, the netmap RX-ring layout)
    stay runnable and bit-exact."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "3", "--warmup", "1",
                        "--cpu-seconds", "0.2", *args],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert line["value"] > 0 and line["parity"]["mismatches"] == 0
    assert line["parity"]["checked_packets"] == line["config"]["packets_per_gpu"]


def test_bench_spawns_ranks_without_torchrun(gpu):
    """`bench.py --gpus 2` with no torchrun environment starts 2 ranks itself
    (the driver's command shape); gloo so both ranks can share cuda:0."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["WC_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2",
                        "--steps", "5", "--warmup", "1", "--packets", "65536"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 2
    assert line["parity"] == {"checked_packets": 2 * 65536, "mismatches": 0}
    assert line["results_allgather"]["ranks_mismatched"] == 0
    assert 0 < line["roofline"]["frac_job"] < 1.5


def test_bench_c5_windowed(gpu):
    """SURVEY C5's 1-GPU shape at reduced size: 2^22 x 1472 B as 4 launches
    over a resident 2^20-packet window, the last window checked in full."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--config", "c5",
                        "--total-packets", str(1 << 22), "--window-packets", str(1 << 20),
                        "--steps", "3", "--warmup", "1", "--cpu-seconds", "0.5"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert line["scaling"] == "strong"
    assert line["config"]["launches_per_step"] == 4
    assert line["config"]["packets_per_gpu"] == 1 << 22
    assert line["parity"] == {"checked_packets": 1 << 20, "mismatches": 0}
    assert line["cpu_baseline"]["best_of"] == 5 and line["cpu_baseline"]["value_1core"] > 0


def test_bench_c5_two_rank_split(gpu):
    """The same strong-scaling split rehearsed at 2 ranks (gloo, sharing
    cuda:0): each rank takes half of the total as 2 launches over its own
    window, checked on every rank."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["WC_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--config", "c5",
                        "--total-packets", str(1 << 22), "--window-packets", str(1 << 20),
                        "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["launches_per_step"] == 2
    assert line["config"]["packets_per_gpu"] == 1 << 21
    assert line["parity"] == {"checked_packets": 2 << 20, "mismatches": 0}


def test_bench_rccl_code_path_one_rank(gpu):
    """bench.py's RCCL (backend "nccl") branch end to end on one GPU: process
    group on cuda:0, barriers, max/sum reductions and the results all-gather
    over RCCL -- the path the driver's 2/4/8-GPU runs take, one rank."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), WC_DIST_FORCE_PG="1", WC_DIST_BACKEND="nccl")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "1", "--steps", "5",
                        "--warmup", "1", "--packets", "65536", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 1 and line["parity"]["mismatches"] == 0
    assert line["results_allgather"]["ranks_mismatched"] == 0

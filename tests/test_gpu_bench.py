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


SMALL_C5 = ["--total-packets", str(1 << 22), "--window-packets", str(1 << 20)]


SMALL_EXTRA = ["--c3-packets", "65536", "--c4-packets", "200000", "--rotate-bytes",
               str(64 << 20), "--extra-seconds", "0.05", "--e2e-packets", "65536",
               "--e2e-reps", "2", "--ring-packets", "65536"]
E2E_CALLS = ("cksum_host", "cksum_ip_udp_host", "rx_verdict_host")


def check_e2e(e2e: dict, ranks: int, n: int = 65536) -> None:
    """The end-to-end object: three host-memory calls x two memory kinds, a
    positive rate against a positive H2D ceiling, every result exact."""
    assert e2e["n_ranks"] == ranks
    assert e2e["h2d_ceiling_GBps"]["pinned"] > 0 and e2e["h2d_ceiling_GBps"]["pageable"] > 0
    assert set(e2e["calls"]) == set(E2E_CALLS)
    for name in E2E_CALLS:
        for kind in ("registered", "pageable"):
            c = e2e["calls"][name][kind]
            assert c["GBps"] > 0 and 0 < c["frac_of_h2d_pinned"] < 2, (name, kind, c)
            assert c["parity"] == {"checked_packets": ranks * 2 * n, "mismatches": 0}, (name, kind)
    assert e2e["rx_frames_ok"] == ranks * n


def test_bench_one_gpu_line(gpu):
    """The driver's line at reduced size: C2 headline, CPU baseline, the C5
    strong-scaling leg (2^22 packets over a 2^20 window here) and the c3 / c4
    objects and C2 rotating cross-check (rotating over >= 64 MiB here)."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "5", "--warmup", "1",
                        "--packets", "65536", "--cpu-seconds", "0.5", *SMALL_C5, *SMALL_EXTRA],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert KEYS <= set(line)
    assert line["n_gpus"] == 1 and line["steps"] == 5 and line["value"] > 0
    assert line["roofline"]["bound"] == "hbm" and 0 < line["roofline"]["frac"] < 1.5
    assert line["cpu_baseline"]["kind"] == "port" and line["cpu_baseline"]["cores"] >= 1
    assert line["parity"]["mismatches"] == 0
    c5 = line["c5"]
    assert c5["scaling"] == "strong" and c5["n_gpus"] == 1 and c5["value"] > 0
    assert "4 launch(es)" in c5["workload"] and 0 < c5["frac_job"] < 1.5
    assert c5["parity"] == {"checked_packets": 3 << 16, "mismatches": 0,
                            "sample": c5["parity"]["sample"]}
    # c3: every size, rotating over ceil(64 MiB / batch) batches, all checked
    c3 = line["c3"]["sizes"]
    assert sorted(int(k) for k in c3) == [64, 256, 576, 1472, 9000]
    for L, e in c3.items():
        K = -(-(64 << 20) // (65536 * int(L)))
        assert e["batches"] == K, (L, e)
        assert e["parity"] == {"checked_packets": K * 65536, "mismatches": 0}, (L, e)
        assert 0 < e["frac"] < 1.5
        assert ("frac_l3_resident" in e) == (K > 1)
    c4 = line["c4"]
    assert c4["parity"] == {"checked_packets": 200000, "mismatches": 0} and c4["frac"] > 0
    rot = line["roofline"]["rotating"]
    assert rot["batches"] == 4 and rot["parity"] == {"checked_packets": 4 * 65536,
                                                      "mismatches": 0}
    assert line["roofline"]["frac_rotating"] == rot["frac"]
    # the shader clock sampled beside each secondary leg (wc_sclk_probe)
    for e in [*c3.values(), c4, rot]:
        assert e["sclk_MHz"] is None or 300 <= e["sclk_MHz"] <= 3500, e
    assert c4["sclk_MHz"] is not None
    check_e2e(line["e2e"], 1)


def test_bench_c3_rotating_line(gpu):
    """`--config c3` rotates over distinct batches (HBM, not the Infinity
    Cache), replays its launches from a hipGraph, checks every batch and
    reports the single-buffer rate beside it."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--config", "c3", "--len", "64",
                        "--steps", "20", "--warmup", "2", "--packets", "65536",
                        "--rotate-bytes", str(16 << 20), "--no-c5", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert line["config"]["batches"] == 4 and line["steps"] % 8 == 0
    assert line["parity"] == {"checked_packets": 4 * 65536, "mismatches": 0}
    assert line["roofline"]["timing"].startswith("hipGraph replay (8 launches per graph)")
    assert 0 < line["roofline"]["frac_l3_resident"] < 1.5


def test_bench_two_ranks_rehearsal(gpu):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, WC_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", str(port), str(ROOT / "bench.py"), "--gpus", "2",
                        "--steps", "5", "--warmup", "1", "--packets", "65536",
                        "--cpu-seconds", "0.3", *SMALL_C5, *SMALL_EXTRA],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["cpu_baseline"]["cores"] >= 1  # rank 0's host cores, at every N
    c5 = line["c5"]  # the strong split: each of 2 ranks takes 2^21 as 2 launches
    assert c5["n_gpus"] == 2 and "2097152 packets per rank as 2 launch(es)" in c5["workload"]
    assert c5["parity"]["checked_packets"] == 2 * (3 << 16) and c5["parity"]["mismatches"] == 0
    assert line["parity"] == {"checked_packets": 2 * 65536, "mismatches": 0}
    assert line["results_allgather"]["ranks_mismatched"] == 0
    assert line["results_allgather"]["bytes_per_rank"] == 2 * 65536
    assert line["c3"]["sizes"]["64"]["parity"]["mismatches"] == 0
    assert line["c4"]["parity"] == {"checked_packets": 2 * 200000, "mismatches": 0}
    check_e2e(line["e2e"], 2)  # both ranks' host calls at once


def test_bench_eight_ranks_rehearsal(gpu):
    """the driver's 8-GPU command shape (`bench.py --gpus
    8`, no torchrun environment: bench starts the 8 ranks itself) rehearsed
    as 8 gloo ranks sharing cuda:0 at reduced sizes.  Every leg of the
    default line runs on every rank: the headline shards, C5's strong split
    (2^22 packets over 8 ranks: 2^19 each, one launch), the c3 / c4 / ring
    legs, the e2e calls on all ranks at once, the results all-gather -- and
    parity is checked on every rank.  The wall time is recorded for
    DESIGN.md section 7."""
    import time
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["WC_DIST_BACKEND"] = "gloo"
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "8",
                        "--steps", "5", "--warmup", "1", "--packets", "65536",
                        "--cpu-seconds", "0.3", *SMALL_C5, *SMALL_EXTRA],
                       capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    wall = time.monotonic() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    line = _last_json(r.stdout)
    print(f"8-rank rehearsal wall time {wall:.1f} s")
    assert line["n_gpus"] == 8 and line["scaling"] == "weak"
    assert line["config"]["parallelism"] == "packet-shard x8"
    assert line["parity"] == {"checked_packets": 8 * 65536, "mismatches": 0}
    g = line["results_allgather"]
    assert g["ranks_mismatched"] == 0 and g["bytes_per_rank"] == 2 * 65536
    c5 = line["c5"]
    assert c5["n_gpus"] == 8 and "524288 packets per rank as 1 launch(es)" in c5["workload"]
    assert c5["parity"]["checked_packets"] == 8 * (3 << 16) and c5["parity"]["mismatches"] == 0
    for L, e in line["c3"]["sizes"].items():
        K = -(-(64 << 20) // (65536 * int(L)))
        assert e["parity"] == {"checked_packets": 8 * K * 65536, "mismatches": 0}, (L, e)
    assert line["c4"]["parity"] == {"checked_packets": 8 * 200000, "mismatches": 0}
    for name in ("rx_mtu", "zrx", "zrx_arp3"):
        assert line["rings"][name]["parity"]["mismatches"] == 0, name
    check_e2e(line["e2e"], 8)
    assert 0 < line["roofline"]["frac_job"] < 1.5


@pytest.mark.parametrize("args", [["--config", "c4", "--packets", "200000"],
                                  ["--config", "c4", "--packets", "200000", "--kind", "payload",
                                   "--headers"],
                                  ["--config", "slots", "--packets", "65536", "--kind", "payload",
                                   "--headers"],
                                  ["--config", "c2", "--packets", "65536", "--kind", "payload"],
                                  ["--config", "c4", "--packets", "200000", "--fused"],
                                  ["--config", "zslots", "--packets", "100000", "--fused"],
                                  ["--config", "c2", "--packets", "65536", "--fused"],
                                  ["--config", "rx", "--packets", "65536"],
                                  ["--config", "zrx", "--packets", "100000"]])
def test_bench_other_configs(gpu, args):
    """The secondary bench lines (C4, payload_cksum, the netmap RX-ring layout)
    stay runnable and bit-exact."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "3", "--warmup", "1",
                        "--cpu-seconds", "0.2", "--no-c5", "--no-extra", *args],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert line["value"] > 0 and line["parity"]["mismatches"] == 0
    # strided batches smaller than 1 GiB rotate over K distinct batches, each checked
    K = line["config"].get("batches", 1)
    assert line["parity"]["checked_packets"] == line["config"]["packets_per_gpu"] * K


def test_bench_spawns_ranks_without_torchrun(gpu):
    """`bench.py --gpus 2` with no torchrun environment starts 2 ranks itself
    (the driver's command shape); gloo so both ranks can share cuda:0."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["WC_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2",
                        "--steps", "5", "--warmup", "1", "--packets", "65536", "--no-c5",
                        "--no-cpu-baseline", "--no-extra", "--batches", "1"],
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
                        "--warmup", "1", "--packets", "65536", "--no-cpu-baseline",
                        "--no-extra", *SMALL_C5],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 1 and line["parity"]["mismatches"] == 0
    assert line["results_allgather"]["ranks_mismatched"] == 0
    assert line["c5"]["parity"]["mismatches"] == 0


def test_c5_full_size_one_gpu(gpu):
    """SURVEY C5 at its full size on one GPU: 2^28 x 1472 B (395 GB) as 8
    windows of 2^25 packets, each regenerated on the device with its own
    seed.  Every packet is checked by the round-trip property -- word 0
    zeroed, ip_cksum computed and stored there, wc_verify_strided must count
    0 bad (the receiver's check, ip4.c:110-115) -- and window 0's checksums
    are compared with the oracle, in 2^22-packet slices."""
    import numpy as np
    import torch

    import warpcore_amd as wc
    from oracle import c_oracle
    from warpcore_amd import synth

    L, win, windows = 1472, 1 << 25, 8
    buf = torch.empty(win * L + 64, dtype=torch.uint8, device=gpu)
    rows = buf[: win * L].view(win, L)
    out = torch.empty(win, dtype=torch.uint16, device=gpu)
    bad = torch.zeros(1, dtype=torch.int64, device=gpu)
    for w in range(windows):
        wc.synth_fill(buf, synth.SEED + 0xC5 * (w + 1), nbytes=win * L)
        rows[:, 0:2] = 0
        wc.cksum_strided(buf, L, L, win, out=out, kind="ip")
        if w == 0:
            sl = 1 << 22
            for s0 in range(0, win, sl):
                hb = buf[s0 * L:(s0 + sl) * L].cpu().numpy()
                want = c_oracle.cksum_strided(hb, L, L, sl, kind=0)
                got = out[s0:s0 + sl].cpu().numpy().view(np.uint16)
                assert np.array_equal(got, want), f"window 0 slice {s0}"
                del hb
        rows[:, 0:2] = out.view(torch.uint8).view(win, 2)
        _, b = wc.verify_strided(buf, L, L, win, kind="ip", out=out)
        bad += b
        torch.cuda.synchronize()
        assert int(b.item()) == 0, f"window {w}: {int(b.item())} packets do not verify"
    assert int(bad.item()) == 0
    del rows, buf, out
    torch.cuda.empty_cache()

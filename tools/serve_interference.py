#!/usr/bin/env python3
"""What the resident server grid costs other work.

C2 (2^20 x 1472 B, device-resident) timed with HIP events on torch's stream
in three states, interleaved round by round:

  none    no server grid on the device (WC_SERVE=0 for the small calls)
  idle    the server's 64 one-wave workgroups resident and polling, no
          requests (started by one small host call, WC_SERVE_IDLE_US long)
  busy    the same grid answering 1-packet host calls from another thread
          back to back while C2 runs

    python tools/serve_interference.py [--rounds 5] [--iters 200]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import warpcore_amd as wc  # noqa: E402
from warpcore_amd import _lib  # noqa: E402

L = 1472


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    os.environ["WC_SERVE_IDLE_US"] = str(60_000_000)  # the watcher stays out of it
    wc.gpu_init(0)
    wc.reload_config()
    dev = torch.device("cuda:0")
    n = 1 << 20
    buf = torch.empty(n * L + 64, dtype=torch.uint8, device=dev)
    wc.synth_fill(buf, 5, nbytes=n * L)
    out = torch.empty(n, dtype=torch.uint16, device=dev)
    torch.cuda.synchronize()  # (before any server grid exists)
    pool = np.random.default_rng(3).integers(0, 256, 1 << 20, dtype=np.uint8)
    wc.host_register(pool)
    off = np.array([64], dtype=np.uint64)
    ln = np.array([1472], dtype=np.uint16)
    want = wc.cksum_host(pool, off, ln)
    stream = torch.cuda.current_stream()

    def c2_us():
        # stream synchronisation only: a device-wide one (torch.cuda.synchronize)
        # waits for the resident server grid to be stopped
        for _ in range(20):
            wc.cksum_strided(buf, L, L, n, out=out)
        stream.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.iters):
            wc.cksum_strided(buf, L, L, n, out=out)
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / args.iters * 1e3

    res = {"none": [], "idle": [], "busy": []}
    calls = []
    for r in range(args.rounds):
        for state in res:
            if state == "none":
                os.environ["WC_SERVE"] = "0"
                wc.reload_config()
                _lib.load().wc_gpu_fini()  # stops a running grid
                wc.gpu_init(0)
                s0 = wc.server_stats()
                assert (wc.cksum_host(pool, off, ln) == want).all()
                assert wc.server_stats()["served"] == s0["served"]  # not the server
                us = c2_us()
            else:
                os.environ["WC_SERVE"] = "1"
                wc.reload_config()
                s0 = wc.server_stats()
                assert (wc.cksum_host(pool, off, ln) == want).all()  # grid up
                assert wc.server_stats()["served"] == s0["served"] + 1
                if state == "idle":
                    us = c2_us()
                else:
                    stop = threading.Event()
                    k = [0]

                    def caller():
                        while not stop.is_set():
                            if not (wc.cksum_host(pool, off, ln) == want).all():
                                raise RuntimeError("server answer differs")
                            k[0] += 1
                    t = threading.Thread(target=caller)
                    t.start()
                    time.sleep(0.01)
                    t0 = time.perf_counter()
                    us = c2_us()
                    dt = time.perf_counter() - t0
                    stop.set()
                    t.join()
                    calls.append(k[0] / max(dt, 1e-9))
                s1 = wc.server_stats()
                assert s1["fallbacks"] == s0["fallbacks"], (s0, s1)
            res[state].append(us)
            print(f"round {r} {state:<5} C2 kernel {us:8.1f} us = {n * L / us / 1e3 / 8000:.4f}",
                  flush=True)
    print("== median over rounds")
    base = statistics.median(res["none"])
    for state, v in res.items():
        m = statistics.median(v)
        print(f"{state:<5} {m:8.1f} us  frac {n * L / m / 1e3 / 8000:.4f}  "
              f"({(m / base - 1) * 100:+.2f} % vs none)", flush=True)
    if calls:
        print(f"busy: {statistics.median(calls):.0f} server calls/s answered during C2", flush=True)
    wc.host_unregister(pool)
    _lib.load().wc_gpu_fini()


if __name__ == "__main__":
    main()

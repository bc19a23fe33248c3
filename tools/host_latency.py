"""Latency of wc_cksum_host on small batches: zero-copy (kernel reads the
registered pool in place) against the pipelined copy path (WC_ZC_BYTES=0).

    python tools/host_latency.py [--reps 300]

Prints one line per (batch, path): median / p10 / p90 microseconds per call,
with the packets spread over a registered 2048-B-slot pool like the socket
backend's (backend_sock.c:145).
"""
import argparse
import os
os.environ.setdefault("WC_TUNING", "1")  # the path knobs set below: the tuning build reads them
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime: torch first)

import warpcore_amd as wc  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--len", type=int, default=1472)
    ap.add_argument("--batches", default="1,8,64,256,1024,4096")
    args = ap.parse_args()
    slot = 2048
    nslots = 8192
    pool = np.random.default_rng(1).integers(0, 256, nslots * slot, dtype=np.uint8)
    wc.host_register(pool)
    try:
        for n in (int(b) for b in args.batches.split(",")):
            offs = (np.random.default_rng(n).permutation(nslots)[:n] * slot).astype(np.uint64)
            lens = np.full(n, args.len, dtype=np.uint16)
            ref = None
            for path, zc in (("zero-copy", str(1 << 30)), ("pipeline", "0")):
                os.environ["WC_ZC_BYTES"] = zc
                wc.reload_config()
                for _ in range(20):
                    out = wc.cksum_host(pool, offs, lens)
                t = []
                for _ in range(args.reps):
                    t0 = time.perf_counter_ns()
                    out = wc.cksum_host(pool, offs, lens)
                    t.append(time.perf_counter_ns() - t0)
                if ref is None:
                    ref = out
                assert (out == ref).all(), "paths disagree"
                t = np.array(t) / 1e3
                gbs = n * args.len / (np.median(t) * 1e3)
                print(f"batch {n:5d} x {args.len} B  {path:9s}  median {np.median(t):8.1f} us"
                      f"  p10 {np.percentile(t, 10):8.1f}  p90 {np.percentile(t, 90):8.1f}"
                      f"  ({gbs:6.2f} GB/s)", flush=True)
    finally:
        os.environ.pop("WC_ZC_BYTES", None)
        wc.host_unregister(pool)


if __name__ == "__main__":
    main()

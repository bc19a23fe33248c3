#!/usr/bin/env python3
"""End-to-end (host memory in, host memory out) checksum rate of the C2 batch
(2^20 x 1472 B) through the host path: chunked hipMemcpyAsync H2D over three
streams per device, the ragged kernel, D2H of the results -- for
  * a page-locked buffer (wc_host_register, e.g. netmap's w->mem): DMA
    straight from it;
  * a pageable buffer: the library first copies each chunk into its pinned
    staging ring (split over its staging workers, WC_STAGE_THREADS).
With --shards G the batch goes through wc_cksum_host_multi over G shard
executors on GPU 0 (the one-thread multi-GPU driver; on a 1-GPU box the
shards share one PCIe link, so this measures the driver, not G links).
Prints one JSON line per case; results checked bit-exact against the oracle.

    python tools/e2e.py [--reps R] [--shards G ...] [--rx]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import warpcore_amd as wc  # noqa: E402
from oracle import c_oracle  # noqa: E402  (checker only)
from warpcore_amd import synth  # noqa: E402


def timed(fn, reps):
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return min(t), sorted(t)[len(t) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--shards", type=int, nargs="*", default=[])
    args = ap.parse_args()
    n, L = 1 << 20, 1472
    wc.gpu_init(0)
    buf = c_oracle.synth(n * L, synth.SEED)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    lens = np.full(n, L, dtype=np.uint16)
    want = c_oracle.cksum_strided(buf, L, L, n, kind=0)
    stage = os.environ.get("WC_STAGE_THREADS", "default")
    for G in [0] + list(args.shards):
        if G:
            wc.gpu_init_multi(devices=[0] * G)
            fn = lambda: wc.cksum_host_multi(buf, offs, lens)  # noqa: E731
        else:
            fn = lambda: wc.cksum_host(buf, offs, lens)  # noqa: E731
        for case in ("pinned", "pageable"):
            if case == "pinned":
                wc.host_register(buf)
            assert np.array_equal(fn(), want), case  # warm-up + check
            best, med = timed(fn, args.reps)
            if case == "pinned":
                wc.host_unregister(buf)
            print(json.dumps({"case": case, "path": f"wc_cksum_host_multi, {G} shards on GPU 0"
                              if G else "wc_cksum_host", "stage_threads": stage,
                              "packets": n, "bytes": n * L, "s_best": best, "s_median": med,
                              "GBps_best": n * L / best / 1e9, "GBps_median": n * L / med / 1e9,
                              "bit_exact": True}), flush=True)
        if G:
            wc._lib.load().wc_gpu_fini()
            wc.gpu_init(0)


if __name__ == "__main__":
    main()

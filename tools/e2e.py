#!/usr/bin/env python3
"""End-to-end (host memory in, host memory out) checksum rate of the C2 batch
(2^20 x 1472 B) through wc_cksum_host: chunked hipMemcpyAsync H2D over three
streams, the ragged kernel, D2H of the results -- for
  * a page-locked buffer (wc_host_register, e.g. netmap's w->mem): DMA
    straight from it;
  * a pageable buffer: the library first memcpy's each chunk into its pinned
    staging ring.
Prints one JSON line per case; results checked bit-exact against the oracle.
"""
import json
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


def main():
    n, L = 1 << 20, 1472
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    wc.gpu_init(0)
    buf = c_oracle.synth(n * L, synth.SEED)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    lens = np.full(n, L, dtype=np.uint16)
    want = c_oracle.cksum_strided(buf, L, L, n, kind=0)
    for case in ("pinned", "pageable"):
        if case == "pinned":
            wc.host_register(buf)
        got = wc.cksum_host(buf, offs, lens)  # warm-up + check
        assert np.array_equal(got, want), case
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            wc.cksum_host(buf, offs, lens)
            t.append(time.perf_counter() - t0)
        if case == "pinned":
            wc.host_unregister(buf)
        best, med = min(t), sorted(t)[len(t) // 2]
        print(json.dumps({"case": case, "packets": n, "bytes": n * L,
                          "s_best": best, "s_median": med,
                          "GBps_best": n * L / best / 1e9, "GBps_median": n * L / med / 1e9,
                          "bit_exact": True}), flush=True)


if __name__ == "__main__":
    main()

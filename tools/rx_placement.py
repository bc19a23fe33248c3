#!/usr/bin/env python3
"""Is the mixed-size RX ring's rate a property of where its buffer lands?

The default bench line's zrx / zrx_arp3 legs read 0.45-0.56 of peak in some
processes and 0.60 / 0.70 in others, every other leg steady (calls q, s).
Each iteration here allocates the 2^21-slot ring afresh (behind a spacer of
random size, so it lands elsewhere), builds the frames, and times the RX
verdicts and the plain ragged payload_cksum of the same datagrams on it:

    python tools/rx_placement.py [--iters 12] [--arp 0] [--launches 200]
"""
from __future__ import annotations

import argparse
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import warpcore_amd as wc  # noqa: E402
from warpcore_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--arp", type=int, default=0)
    ap.add_argument("--launches", type=int, default=200)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    wc.gpu_init(0)
    stream = torch.cuda.current_stream()
    n, slot = 1 << 21, 2048
    ip_lens = synth.zipf_lengths(n)
    rng = np.random.default_rng(11)
    rows = []

    def timed(fn):
        for _ in range(20):
            fn()
        stream.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.launches):
            fn()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / args.launches * 1e3

    for it in range(args.iters):
        spacer = torch.empty(int(rng.integers(1, 512)) << 20, dtype=torch.uint8, device=dev)
        buf = torch.empty(n * slot + 64, dtype=torch.uint8, device=dev)
        wc.synth_fill(buf, 1, nbytes=n * slot)
        f_off, f_len = synth.make_rx_ring(buf, n, ip_lens)
        if args.arp:
            sel = torch.from_numpy(f_off[::args.arp].astype(np.int64)).to(dev)
            buf[sel + 12] = 0x08
            buf[sel + 13] = 0x06
        d_off = torch.from_numpy(f_off).to(dev)
        d_len = torch.from_numpy(f_len).to(dev)
        ip_off = torch.from_numpy((f_off + np.uint64(14)).astype(np.uint64)).to(dev)
        ip_len = torch.from_numpy(ip_lens).to(dev)
        out = torch.empty(n, dtype=torch.uint8, device=dev)
        out16 = torch.empty(n, dtype=torch.uint16, device=dev)
        drops = torch.zeros(1, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        rx = timed(lambda: wc.rx_verdict_ragged(buf, d_off, d_len, out=out, check=False,
                                                drops=drops))
        pay = timed(lambda: wc.cksum_ragged(buf, ip_off, ip_len, out=out16, kind="payload",
                                            check=False))
        va = buf.data_ptr()
        rows.append((rx, pay))
        print(f"iter {it:2d} ring at {va:#x} (mod 2 MiB {va % (2 << 20):#x}, mod 1 GiB "
              f"{va % (1 << 30):#x}): rx {rx:7.1f} us  payload {pay:7.1f} us", flush=True)
        del buf, d_off, d_len, ip_off, ip_len, out, out16, drops, spacer
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    rxs = [r for r, _ in rows]
    pays = [p for _, p in rows]
    print(f"rx      min {min(rxs):.1f} median {statistics.median(rxs):.1f} max {max(rxs):.1f} us")
    print(f"payload min {min(pays):.1f} median {statistics.median(pays):.1f} max {max(pays):.1f} us")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-tile phase timing of k_rx_verdict on the mixed-size ring (diagnostic).

    WC_LIB=tools/libwc_stamps.so python tools/rx_stamps.py [--config zrx|rx]

Needs a library built with -DWC_DIAG_STAMPS (wc_k_rx.hip): lane 0 of every
tile stores the 100-MHz wall clock at the tile's start (s0), once the header
loads are issued (s1: metadata arrived), at the end of the header parse (s2),
after the stream and payload arithmetic (s3) and after the verdict store
(s4), plus the tile's stream length in 16-B slots and the wave's hardware ids.
Prints the phase durations (10-ns ticks) and the wave residency picture.
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
os.environ.setdefault("WC_TUNING", "0")

import torch  # noqa: E402

import warpcore_amd as wc  # noqa: E402
from warpcore_amd import _lib, synth  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="zrx", choices=["zrx", "rx"])
    ap.add_argument("--runs", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    wc.gpu_init(0)
    n = 1 << 21 if args.config == "zrx" else 1 << 20
    ip_lens = synth.zipf_lengths(n) if args.config == "zrx" else np.full(n, 1500, np.uint16)
    buf = torch.empty(n * 2048 + 64, dtype=torch.uint8, device=dev)
    wc.synth_fill(buf, 1, nbytes=n * 2048)
    f_off, f_len = synth.make_rx_ring(buf, n, ip_lens)
    d_off, d_len = torch.from_numpy(f_off).to(dev), torch.from_numpy(f_len).to(dev)
    out = torch.empty(n, dtype=torch.uint8, device=dev)
    lib = _lib.active()
    fn = lib.wc_diag_rx_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(args.runs):
        ev0.record()
        wc.rx_verdict_ragged(buf, d_off, d_len, out=out, check=False)
        ev1.record()
    torch.cuda.synchronize()
    print(f"last launch {ev0.elapsed_time(ev1) * 1e3:.1f} us (events, includes the launch)")
    tiles = min((n + 63) // 64, 1 << 16)
    st = np.zeros(tiles * 8, dtype=np.uint32)
    assert fn(st.ctypes.data, st.size) == 0
    st = st.reshape(tiles, 8).astype(np.int64)
    s = st[:, :5]
    base = s[:, 0].min()
    s = s - base
    T = st[:, 5]
    spec = s[:, 3] > 0
    d = {
        "meta (s1-s0)": s[:, 1] - s[:, 0],
        "hdr+parse (s2-s1)": s[:, 2] - s[:, 1],
        "stream+sum (s3-s2)": s[:, 3] - s[:, 2],
        "store (s4-s3)": s[:, 4] - s[:, 3],
        "tile (s4-s0)": s[:, 4] - s[:, 0],
    }
    print(f"tiles {tiles}, with stream {int(spec.sum())}, span {s[:, 4].max() / 100:.1f} us")
    for k, v in d.items():
        v = v[spec]
        print(f"  {k:22s} median {np.median(v) / 100:7.2f} us  p10 {np.percentile(v, 10) / 100:7.2f}"
              f"  p90 {np.percentile(v, 90) / 100:7.2f}  mean {v.mean() / 100:7.2f}")
    rows = (T[spec] + 63) // 64
    print(f"  stream rows per tile: median {np.median(rows):.0f} mean {rows.mean():.1f}")
    per_row = (s[spec, 3] - s[spec, 2]) / np.maximum(rows, 1) / 100
    print(f"  stream time per row: median {np.median(per_row) * 1e3:.0f} ns")
    # starts over time: how many tiles start per 1-us bin, and concurrent tiles
    starts, ends = s[:, 0], s[:, 4]
    span = int(ends.max()) + 1
    edges = np.arange(0, span + 100, 100)
    live = np.zeros(len(edges))
    for a, b in zip(starts, ends):
        live[int(a) // 100: int(b) // 100 + 1] += 1
    print("  concurrent tiles per 1-us bin (every 8th):",
          " ".join(str(int(x)) for x in live[::8]))
    first_end = np.sort(ends)[:5] / 100
    print(f"  first tile ends at {first_end} us; last tile starts at {starts.max() / 100:.1f} us")
    np.save(ROOT / "gpurun_out" / f"rx_stamps_{args.config}.npy", st)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Measurement tool: HBM read rate per lane pattern (tools/pattern_probe.hip),
interleaved rounds in one process, HIP events on the launch stream.

    python tools/pattern_probe.py [--gb 2] [--rounds 5] [--iters 20]
"""
import argparse
import ctypes
import statistics
import subprocess
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent


def lib():
    so = ROOT / "tools" / "libpattern_probe.so"
    src = ROOT / "tools" / "pattern_probe.hip"
    if not so.exists() or so.stat().st_mtime < src.stat().st_mtime:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC",
                        "-shared", "-o", str(so), str(src)], check=True)
    l = ctypes.CDLL(str(so))
    l.probe_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    return l


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=2.0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    L = lib()
    nbytes = int(args.gb * 1e9) // 8192 * 8192
    buf = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda")
    sink = torch.zeros(64, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    cases = [(w, k, sh) for (w, k) in [(64, 4), (16, 4), (8, 4), (4, 4), (4, 2), (8, 2),
                                       (16, 2), (2, 4)]
             for sh in (0, 1, 2, 4)]
    t = {c: [] for c in cases}
    for _ in range(args.rounds):
        for w, k, sh in cases:
            fn = lambda: L.probe_read(buf.data_ptr(), nbytes, w, k, sink.data_ptr(),  # noqa
                                      st.cuda_stream, sh)
            assert fn() == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.iters):
                fn()
            e1.record(st)
            e1.synchronize()
            t[(w, k, sh)].append(e0.elapsed_time(e1) / args.iters)
    for (w, k, sh), ts in t.items():
        med = statistics.median(ts)
        print(f"W={w:<3} K={k} shift={16 * sh:<3}B  {med * 1e3:8.1f} us  "
              f"{nbytes / med / 1e6:8.1f} GB/s  "
              f"{nbytes / med / 1e6 / 80:5.1f}% of 8 TB/s", flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""C5 window vs C2, same thermal state (second probe).

The first probe (tools/c5_probe.sh, profiles/c5probe_r05_*) found the C5
window's PMC counters scale with C2's bytes except the cycle counters (about
20x the cycles for 32x the bytes), i.e. the shader clock ran lower during the
49-GB launches.  This tool runs, interleaved round by round and each phase
after its own warm-up:

  c2        the 2^20 x 1472 B batch, launches back to back
  c5        the 2^25-packet (49 GB) window, one launch each
  c5split   the same window as 32 launches of 2^20-packet slices
  c5cap<K>  the window on a grid capped at K blocks per CU (grid-stride)

timing each with HIP events and sampling the shader clock beside it with a
one-wave probe kernel on a second stream (tools/clock_probe.hip).

    python tools/c5_clock.py [--rounds 3] [--phase-ms 60] [--caps 8,16]
"""
from __future__ import annotations

import argparse
import ctypes
import os
os.environ.setdefault("WC_TUNING", "1")  # the path knobs set below: the tuning build reads them
import statistics
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import warpcore_amd as wc  # noqa: E402
from warpcore_amd import _lib  # noqa: E402

L = 1472


def probe_lib():
    so = ROOT / "tools" / "libclock_probe.so"
    src = ROOT / "tools" / "clock_probe.hip"
    if not so.exists() or so.stat().st_mtime < src.stat().st_mtime:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC",
                        "-shared", "-o", str(so), str(src)], check=True)
    lib = ctypes.CDLL(str(so))
    lib.clock_probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64,
                                       ctypes.c_void_p]
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--phase-ms", type=float, default=60.0)
    ap.add_argument("--caps", default="8,16")
    ap.add_argument("--window", type=int, default=1 << 25)
    args = ap.parse_args()

    dev = torch.device("cuda:0")
    wc.gpu_init(0)
    lib = _lib.load()
    plib = probe_lib()
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    pstream = torch.cuda.Stream()

    win = args.window
    small = 1 << 20
    buf = torch.empty(win * L + 64, dtype=torch.uint8, device=dev)
    wc.synth_fill(buf, 11, nbytes=win * L)
    c2buf = torch.empty(small * L + 64, dtype=torch.uint8, device=dev)
    wc.synth_fill(c2buf, 12, nbytes=small * L)
    out = torch.empty(win, dtype=torch.uint16, device=dev)
    samples = torch.zeros(2 * 200000, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()

    def launch(ptr, n, o):
        rc = lib.wc_cksum_strided(ctypes.c_void_p(ptr), L, L, n, ctypes.c_void_p(o), 0, sp)
        if rc != 0:
            raise RuntimeError(f"wc_cksum_strided rc {rc}")

    base = buf.data_ptr()
    optr = out.data_ptr()
    phases = {
        "c2": (lambda: launch(c2buf.data_ptr(), small, optr), small * L, None),
        "c5": (lambda: launch(base, win, optr), win * L, None),
        "c5split": (lambda: [launch(base + k * small * L, small, optr + 2 * k * small)
                             for k in range(win // small)], win * L, None),
    }
    for c in [int(x) for x in args.caps.split(",") if x]:
        phases[f"c5cap{c}"] = (lambda: launch(base, win, optr), win * L, c)

    def set_cap(c):
        if c is None:
            os.environ.pop("WC_BLOCKS_PER_CU", None)
        else:
            os.environ["WC_BLOCKS_PER_CU"] = str(c)
        wc.reload_config()

    res = {k: [] for k in phases}
    clk = {k: [] for k in phases}
    for r in range(args.rounds):
        for name, (fn, nbytes, cap) in phases.items():
            set_cap(cap)
            t_w = time.perf_counter()
            while (time.perf_counter() - t_w) * 1e3 < 30:  # warm-up (untimed)
                fn()
                torch.cuda.synchronize()
            # one calibration call, then enough calls for the phase length
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            e1.synchronize()
            per = e0.elapsed_time(e1)
            iters = max(1, int(args.phase_ms / max(per, 1e-3)))
            ns = int(min(200000, args.phase_ms * 1e3 / 20 + 50))  # one sample per 20 us
            samples.zero_()
            torch.cuda.synchronize()
            rc = plib.clock_probe_launch(ctypes.c_void_p(samples.data_ptr()), ns, 2000,
                                         ctypes.c_void_p(pstream.cuda_stream))
            assert rc == 0, rc
            e0.record(stream)
            for _ in range(iters):
                fn()
            e1.record(stream)
            e1.synchronize()
            ms = e0.elapsed_time(e1) / iters
            torch.cuda.synchronize()
            s = samples[: 2 * ns].view(ns, 2).cpu()
            dt = (s[1:, 0] - s[:-1, 0]).double()
            dc = (s[1:, 1] - s[:-1, 1]).double()
            ok = dt > 0
            mhz = (dc[ok] / dt[ok] * 100.0).tolist()  # wall clock = 100 MHz
            mhz.sort()
            med = mhz[len(mhz) // 2] if mhz else float("nan")
            lo = mhz[len(mhz) // 20] if mhz else float("nan")
            res[name].append(ms)
            clk[name].append(med)
            print(f"round {r} {name:<10} {ms * 1e3:10.1f} us/call  {nbytes / ms / 1e6:7.1f} GB/s "
                  f"= {nbytes / ms / 1e6 / 8000:.4f}  sclk median {med:6.0f} MHz (p5 {lo:6.0f})"
                  f"  {iters} calls", flush=True)
    set_cap(None)
    print("== median over rounds")
    for name, (fn, nbytes, cap) in phases.items():
        ms = statistics.median(res[name])
        print(f"{name:<10} {ms * 1e3:10.1f} us/call  {nbytes / ms / 1e6 / 8000:.4f} of 8 TB/s  "
              f"sclk {statistics.median(clk[name]):6.0f} MHz", flush=True)
    # parity of the last split round against the one-launch results: identical
    # bytes, identical checksums (a cheap self-check; the oracle checks live in
    # tests/)
    launch(base, win, optr)
    ref = out[:: 4097].clone()
    for k in range(win // small):
        launch(base + k * small * L, small, optr + 2 * k * small)
    assert torch.equal(ref, out[:: 4097]), "split launches differ from one launch"
    print("split == one launch: ok", flush=True)


if __name__ == "__main__":
    main()

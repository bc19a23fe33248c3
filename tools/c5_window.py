#!/usr/bin/env python3
"""C5-window experiments: why does one launch over a
49 GB window (2^25 x 1472 B, the per-GPU work of the 8-GPU point) run a few
points below C2 (2^20 x 1472 B) on the same kernel?

    python tools/c5_window.py [--windows 1048576,8388608,33554432]
                              [--allocs torch,hip,contig] [--variants spec;spec]
                              [--rounds R] [--iters I]

Each window size is allocated once per allocator -- torch's caching
allocator (as bench.py does), plain hipMalloc, and hipExtMallocWithFlags with
hipDeviceMallocContiguous (one physically contiguous range: the page tables
can then describe it with large fragments) -- filled with the same splitmix64
bytes, and timed with HIP events on the launch stream, every (alloc, window,
variant) interleaved round by round.  Results of every case are compared with
the first case of the same window (bit-identical bytes, so bit-identical
checksums).  Variants are env strings (WC_VARIANT needs the tuning build).
"""
from __future__ import annotations

import argparse
import ctypes
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

if "WC_VARIANT" in " ".join(sys.argv) or "WC_VARIANT" in os.environ:
    os.environ.setdefault("WC_TUNING", "1")

import torch  # noqa: E402

import warpcore_amd as wc  # noqa: E402
from warpcore_amd import _lib  # noqa: E402

L = 1472
HIP_CONTIG = 0x4  # hipDeviceMallocContiguous (hip_runtime_api.h)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", default=f"{1 << 20},{1 << 23},{1 << 25}")
    ap.add_argument("--allocs", default="torch,hip,contig")
    ap.add_argument("--variants", default="default")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=0,
                    help="launches per timing (0: about 0.2 s worth)")
    ap.add_argument("--warm-ms", type=float, default=200.0)
    args = ap.parse_args()

    dev = torch.device("cuda:0")
    wc.gpu_init(0)
    lib = _lib.load()
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t,
                                          ctypes.c_uint]
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)

    windows = [int(w) for w in args.windows.split(",")]
    allocs = args.allocs.split(",")
    variants = [("" if v.strip() == "default" else v.strip())
                for v in args.variants.split(";") if v.strip()]
    base_env = {k: os.environ.get(k) for k in
                {kv.split("=", 1)[0] for v in variants for kv in v.split()}}

    def apply(spec):
        for k, v in base_env.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        for kv in spec.split():
            k, v = kv.split("=", 1)
            os.environ[k] = v
        wc.reload_config()

    bufs = {}
    keep = []
    for w in windows:
        nbytes = w * L + 64
        for a in allocs:
            if a == "torch":
                t = torch.empty(nbytes, dtype=torch.uint8, device=dev)
                keep.append(t)
                ptr = t.data_ptr()
            else:
                p = ctypes.c_void_p()
                rc = (hip.hipMalloc(ctypes.byref(p), nbytes) if a == "hip" else
                      hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, HIP_CONTIG))
                if rc != 0 or not p.value:
                    print(f"!! {a} alloc of {nbytes} B failed: rc {rc}", flush=True)
                    continue
                ptr = p.value
            rc = lib.wc_synth_fill(ctypes.c_void_p(ptr), w * L, 7, sp)
            assert rc == 0, rc
            out = torch.empty(w, dtype=torch.uint16, device=dev)
            bufs[(a, w)] = (ptr, out)
            print(f"alloc {a:<6} window {w:>9} packets ({w * L / 1e9:6.2f} GB) at "
                  f"{ptr:#x}", flush=True)
    torch.cuda.synchronize()

    def launch(ptr, out, w):
        rc = lib.wc_cksum_strided(ctypes.c_void_p(ptr), L, L, w, ctypes.c_void_p(out.data_ptr()),
                                  0, sp)
        if rc != 0:
            raise RuntimeError(f"wc_cksum_strided rc {rc}")

    times = {}
    ref = {}
    for r in range(args.rounds):
        for (a, w), (ptr, out) in bufs.items():
            for v in variants:
                apply(v)
                t_w = time.perf_counter()
                while (time.perf_counter() - t_w) * 1e3 < args.warm_ms:
                    launch(ptr, out, w)
                    torch.cuda.synchronize()
                iters = args.iters or max(2, int(0.2 / (w * L / 7.4e12)))
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(iters):
                    launch(ptr, out, w)
                e1.record(stream)
                e1.synchronize()
                ms = e0.elapsed_time(e1) / iters
                times.setdefault((a, w, v), []).append(ms)
                if r == 0:
                    res = out[: 1 << 20].cpu()
                    if w not in ref:
                        ref[w] = res
                    elif not torch.equal(ref[w], res):
                        print(f"!! {a} {w} {v!r}: results differ", flush=True)
                print(f"  round {r} {a:<6} {w:>9} {v or 'default':<28} {ms * 1e3:10.1f} us "
                      f"{w * L / ms / 1e6 / 8000 * 100:6.2f} %", flush=True)
    apply("")
    print("== median over rounds (frac of 8 TB/s)")
    for (a, w, v), ts in times.items():
        med = statistics.median(ts)
        print(f"{a:<6} {w:>9} {v or 'default':<28} {med * 1e3:10.1f} us  "
              f"{w * L / med / 1e6:7.1f} GB/s  {w * L / med / 1e6 / 8000:.4f}", flush=True)
    for (a, w), (ptr, out) in bufs.items():
        if a != "torch":
            hip.hipFree(ctypes.c_void_p(ptr))


if __name__ == "__main__":
    main()

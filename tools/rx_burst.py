#!/usr/bin/env python3
"""The mixed-size RX ring timed in bursts of back-to-back launches.

tune.py times 20 launches between synchronisations and reads the mixed ring
at 112 us; tools/rx_placement.py times 200 and reads 121 us; the bench leg
times ~2000 and read 112-149 us from process to process.  Per burst length,
interleaved round by round: the RX verdicts (ADAPT default, and the plain HT
kernel without the tally), the plain ragged payload_cksum of the same
datagrams, and C2, each with the shader clock sampled beside it by a one-wave
probe on a second stream (tools/clock_probe.hip).

    python tools/rx_burst.py [--bursts 20,200,2000] [--rounds 3]
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

import numpy as np  # noqa: E402
import torch  # noqa: E402

import warpcore_amd as wc  # noqa: E402
from warpcore_amd import synth  # noqa: E402


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
    ap.add_argument("--bursts", default="20,200,2000")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--c4", action="store_true", help="add C4 (2^24 Zipf packed, 4 GB)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    wc.gpu_init(0)
    plib = probe_lib()
    stream = torch.cuda.current_stream()
    pstream = torch.cuda.Stream()
    n, slot = 1 << 21, 2048
    ip_lens = synth.zipf_lengths(n)
    buf = torch.empty(n * slot + 64, dtype=torch.uint8, device=dev)
    wc.synth_fill(buf, 1, nbytes=n * slot)
    f_off, f_len = synth.make_rx_ring(buf, n, ip_lens)
    d_off = torch.from_numpy(f_off).to(dev)
    d_len = torch.from_numpy(f_len).to(dev)
    ip_off = torch.from_numpy((f_off + np.uint64(14)).astype(np.uint64)).to(dev)
    ip_len = torch.from_numpy(ip_lens).to(dev)
    out = torch.empty(n, dtype=torch.uint8, device=dev)
    out16 = torch.empty(n, dtype=torch.uint16, device=dev)
    drops = torch.zeros(1, dtype=torch.int64, device=dev)
    c2n, L = 1 << 20, 1472
    c2 = torch.empty(c2n * L + 64, dtype=torch.uint8, device=dev)
    wc.synth_fill(c2, 3, nbytes=c2n * L)
    c2out = torch.empty(c2n, dtype=torch.uint16, device=dev)
    samples = torch.zeros(2 * 200000, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()

    def rx():
        wc.rx_verdict_ragged(buf, d_off, d_len, out=out, check=False, drops=drops)

    def pay():
        wc.cksum_ragged(buf, ip_off, ip_len, out=out16, kind="payload", check=False)

    def c2fn():
        wc.cksum_strided(c2, L, L, c2n, out=c2out)

    cases = [("rx ADAPT", rx, ""), ("rx HT, no tally", rx, "WC_RX_ADAPT=0"),
             ("payload", pay, ""), ("C2", c2fn, "")]
    if args.c4:  # C4: 2^24 Zipf packets packed (the dense seg path)
        c4_lens = synth.zipf_lengths(1 << 24)
        c4_offs = synth.packed_offsets(c4_lens)
        span = int(c4_lens.astype(np.uint64).sum())
        c4buf = torch.empty(span + 64, dtype=torch.uint8, device=dev)
        wc.synth_fill(c4buf, 4, nbytes=span)
        c4_off = torch.from_numpy(c4_offs).to(dev)
        c4_len = torch.from_numpy(c4_lens).to(dev)
        c4out = torch.empty(1 << 24, dtype=torch.uint16, device=dev)

        def c4fn():
            wc.cksum_ragged(c4buf, c4_off, c4_len, out=c4out, check=False)
        cases.append(("C4", c4fn, ""))
    bursts = [int(b) for b in args.bursts.split(",")]
    res, clk = {}, {}

    def apply(spec):
        os.environ.pop("WC_RX_ADAPT", None)
        for kv in spec.split():
            k, v = kv.split("=", 1)
            os.environ[k] = v
        wc.reload_config()

    for r in range(args.rounds):
        for b in bursts:
            for name, fn, spec in cases:
                apply(spec)
                for _ in range(20):  # warm, in bursts with gaps
                    fn()
                torch.cuda.synchronize()
                time.sleep(0.05)
                per = {"C2": 0.21, "C4": 0.62}.get(name, 0.12)  # ms per launch, rough
                ns = int(min(200000, b * per * 1e3 / 20 + 100))
                samples.zero_()
                torch.cuda.synchronize()
                plib.clock_probe_launch(ctypes.c_void_p(samples.data_ptr()), ns, 2000,
                                        ctypes.c_void_p(pstream.cuda_stream))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(b):
                    fn()
                e1.record(stream)
                e1.synchronize()
                us = e0.elapsed_time(e1) / b * 1e3
                pstream.synchronize()
                s = samples[: 2 * ns].view(ns, 2).cpu()
                dt = (s[1:, 0] - s[:-1, 0]).double()
                dc = (s[1:, 1] - s[:-1, 1]).double()
                ok = dt > 0
                mhz = sorted((dc[ok] / dt[ok] * 100.0).tolist())
                med = mhz[len(mhz) // 2] if mhz else float("nan")
                res.setdefault((name, b), []).append(us)
                clk.setdefault((name, b), []).append(med)
                print(f"round {r} burst {b:5d} {name:<16} {us:8.1f} us  sclk {med:6.0f} MHz",
                      flush=True)
    apply("")
    print("== medians")
    for (name, b), v in res.items():
        print(f"burst {b:5d} {name:<16} {statistics.median(v):8.1f} us  "
              f"sclk {statistics.median(clk[(name, b)]):6.0f} MHz", flush=True)


if __name__ == "__main__":
    main()

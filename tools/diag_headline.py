#!/usr/bin/env python3
"""Where the headline's whole-job time goes beyond its kernels (measurement
tool, not product code).

bench.py times 20 C2 launches between two barrier + synchronize brackets; the
driver's line showed 6 us per step between that wall time and the HIP-event
kernel time.  This repeats the same timed region R times in one process, for
several ways of issuing and waiting, interleaved round by round:

  py       bench.py's loop: wc.cksum_strided() per step (Python checks + ctypes)
  raw      the C ABI called straight through ctypes with precomputed arguments
  graph    the 20 launches captured once in a hipGraph, one replay
  *+spin   the same, but the host spins on the last event before synchronize

and, for each, splits the wall time: t0 -> the first event completes on the
GPU (spinning on it right after the first launch; the launches behind it queue
while kernel 1 runs), the kernels (event to event), last event -> sync return.

    python tools/diag_headline.py [--rounds R] [--steps K]
"""
import argparse
import ctypes
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import warpcore_amd as wc  # noqa: E402
from warpcore_amd import _lib, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    wc.gpu_init(0)
    n, L = 1 << 20, 1472
    buf = torch.empty(n * L + 64, dtype=torch.uint8, device=dev)
    wc.synth_fill(buf, synth.SEED, nbytes=n * L)
    out = torch.empty(n, dtype=torch.uint16, device=dev)
    stream = torch.cuda.current_stream(dev)
    lib = _lib.load()
    fn = lib.wc_cksum_strided
    a = (ctypes.c_void_p(buf.data_ptr()), ctypes.c_uint64(L), ctypes.c_uint16(L),
         ctypes.c_uint64(n), ctypes.c_void_p(out.data_ptr()), ctypes.c_int(0),
         ctypes.c_void_p(stream.cuda_stream))

    def py_step():
        wc.cksum_strided(buf, L, L, n, out=out, kind="ip")

    def raw_step():
        rc = fn(*a)
        if rc:
            raise RuntimeError(rc)

    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(args.steps):
            py_step()
    torch.cuda.synchronize()

    def run(how, spin, first_probe):
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(stream)
        t_first = None
        if how == "graph":
            g.replay()
            if first_probe:
                while not ev0.query():
                    pass
                t_first = time.perf_counter()
        else:
            step = py_step if how == "py" else raw_step
            step()
            if first_probe:
                while not ev0.query():
                    pass
                t_first = time.perf_counter()
            for _ in range(args.steps - 1):
                step()
        t_enq = time.perf_counter()
        ev1.record(stream)
        if spin:
            while not ev1.query():
                pass
        t_done = time.perf_counter()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        k_ms = ev0.elapsed_time(ev1)
        return {"wall_ms": (t1 - t0) * 1e3, "kern_ms": k_ms, "enq_ms": (t_enq - t0) * 1e3,
                "first_ms": None if t_first is None else (t_first - t0) * 1e3,
                "spin_to_sync_ms": (t1 - t_done) * 1e3}

    cases = [(h, s, p) for h in ("py", "raw", "graph") for s in (False, True) for p in (False, True)]
    res = {c: [] for c in cases}
    for _ in range(5):  # warm: clocks up
        for c in cases:
            run(*c)
    for _ in range(args.rounds):
        for c in cases:
            res[c].append(run(*c))
    rows = []
    for (h, s, p), rs in res.items():
        gap = [r["wall_ms"] - r["kern_ms"] for r in rs]
        row = {"issue": h, "spin": s, "first_probe": p,
               "gap_us_med": statistics.median(gap) * 1e3, "gap_us_min": min(gap) * 1e3,
               "gap_us_max": max(gap) * 1e3,
               "kern_us_per_step_med": statistics.median(r["kern_ms"] for r in rs) * 1e3 / args.steps,
               "enq_us_med": statistics.median(r["enq_ms"] for r in rs) * 1e3,
               "sync_after_spin_us_med": statistics.median(r["spin_to_sync_ms"] for r in rs) * 1e3}
        if p:
            row["t0_to_first_event_us_med"] = statistics.median(r["first_ms"] for r in rs) * 1e3
        rows.append(row)
        print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in row.items()}),
              flush=True)
    if args.json:
        Path(args.json).write_text(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()

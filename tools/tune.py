#!/usr/bin/env python3
"""Interleaved A/B timing of kernel variants in ONE process (guide rule 24).

    python tools/tune.py [--config c2|c3|c4] [--len L] [--rounds R] [--iters I]
                         [--variants spec;spec;...] [--ceiling]

A variant spec is a comma-free env string, e.g.
"WC_SHAPE=32,3,1 WC_NT=1 WC_BLOCKS_PER_CU=4".  Each round runs every variant
for I launches timed with HIP events on the launch stream; the table reports
median and best GB/s (payload bytes / kernel time) per variant.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

# The WC_* path knobs (and WC_VARIANT / WC_DIAG_NOLOAD) are read by the
# tuning build alone (-DWC_TUNING, libwccksum_tune.so): every variant runs on
# it, the default included.
os.environ.setdefault("WC_TUNING", "1")

import numpy as np  # noqa: E402
import torch  # noqa: E402

import warpcore_amd as wc  # noqa: E402
from warpcore_amd import synth  # noqa: E402


def stream_lib():
    so = ROOT / "tools" / "libstream_ceiling.so"
    src = ROOT / "tools" / "stream_ceiling.hip"
    if not so.exists() or so.stat().st_mtime < src.stat().st_mtime:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC",
                        "-shared", "-o", str(so), str(src)], check=True)
    lib = ctypes.CDLL(str(so))
    lib.stream_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    lib.tile_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                              ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    lib.slot_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                              ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                              ctypes.c_void_p, ctypes.c_void_p]
    lib.line_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                              ctypes.c_void_p, ctypes.c_void_p]
    return lib


def touched_lines(offs: np.ndarray, lens: np.ndarray, line: int = 128) -> np.ndarray:
    """uint32 indices of every `line`-byte line the ranges [off, off + len)
    touch, in range order (each line once per range)."""
    offs = offs.astype(np.int64)
    lens = lens.astype(np.int64)
    keep = lens > 0
    first = offs[keep] // line
    last = (offs[keep] + lens[keep] - 1) // line
    cnt = last - first + 1
    start = np.repeat(np.cumsum(cnt) - cnt, cnt)
    return (np.repeat(first, cnt) + (np.arange(int(cnt.sum())) - start)).astype(np.uint32)


def time_it(fn, iters, stream):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(iters):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters  # ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--len", type=int, default=1472)
    ap.add_argument("--packets", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="")
    ap.add_argument("--ceiling", action="store_true")
    ap.add_argument("--json", default="")
    ap.add_argument("--verbose", action="store_true", help="print every round's time")
    ap.add_argument("--warm-ms", type=float, default=30.0,
                    help="run each variant this long (untimed) before its timed launches, "
                         "so a small batch is timed at ramped clocks")
    ap.add_argument("--kind", default="ip", choices=["ip", "payload"])
    ap.add_argument("--offset", type=int, default=0, help="byte offset of packet 0 (c2/c3)")
    ap.add_argument("--stride", type=int, default=0, help="packet stride (c2/c3; default len)")
    ap.add_argument("--fused", action="store_true",
                    help="fused IPv4 header + payload_cksum pass (wc_cksum_ip_udp_*)")
    ap.add_argument("--headers", action="store_true",
                    help="well-formed IPv4 / IPv6 UDP headers (synth.stamp_udp_headers)")
    ap.add_argument("--rotate-bytes", type=int, default=0,
                    help="c2/c3: rotate the launches over ceil(B / batch) distinct buffers "
                         "(HBM, not the 256 MiB Infinity Cache)")
    ap.add_argument("--rx-arp", type=int, default=0,
                    help="rx / zrx: every K-th frame an ARP frame (no UDP check)")
    ap.add_argument("--rx-packed", action="store_true",
                    help="rx / zrx: the frames back to back (C4's layout) instead of one per "
                         "2048-B slot")
    ap.add_argument("--ragged", action="store_true",
                    help="c2/c3 through the ragged entry point (offset/length arrays)")
    args = ap.parse_args()

    dev = torch.device("cuda:0")
    wc.gpu_init(0)
    stream = torch.cuda.current_stream()
    if args.config in ("rx", "zrx"):
        # netmap RX ring of well-formed UDP frames (bench.py --config rx / zrx);
        # --rx-arp K turns every K-th frame into an ARP frame (no UDP check)
        n = args.packets if args.packets != (1 << 20) or args.config == "rx" else 1 << 21
        ip_lens = (np.full(n, args.len + 28, dtype=np.uint16) if args.config == "rx"
                   else synth.zipf_lengths(n))
        buf = torch.empty(n * 2048 + 64, dtype=torch.uint8, device=dev)
        wc.synth_fill(buf, 1, nbytes=n * 2048)
        f_off, f_len = synth.make_rx_ring(buf, n, ip_lens, packed=args.rx_packed)
        if args.rx_arp:
            sel = torch.from_numpy(f_off[::args.rx_arp].astype(np.int64)).to(dev)
            buf[sel + 12] = 0x08
            buf[sel + 13] = 0x06
        d_off, d_len = torch.from_numpy(f_off).to(dev), torch.from_numpy(f_len).to(dev)
        nbytes = int(f_len.astype(np.uint64).sum())
        out = torch.empty(n, dtype=torch.uint8, device=dev)
        drops = torch.zeros(1, dtype=torch.int64, device=dev)
        run = lambda: wc.rx_verdict_ragged(buf, d_off, d_len, out=out, check=False,  # noqa: E731
                                           drops=drops)
    elif args.config in ("c4", "c4r", "zslots"):
        # c4: Zipf lengths packed; zslots: the same lengths in 2048-B slots at
        # +14 (a netmap RX ring of mixed sizes)
        n = args.packets if args.packets != (1 << 20) else (1 << 21 if args.config == "zslots"
                                                             else 1 << 24)
        lens = synth.zipf_lengths(n)
        if args.config in ("c4", "c4r"):
            offs = synth.packed_offsets(lens)
            span = int(lens.astype(np.uint64).sum())
            if args.config == "c4r":  # the same packets listed in random order
                perm = np.random.default_rng(5).permutation(n)
                offs, lens = offs[perm].copy(), lens[perm].copy()
        else:
            offs = (np.arange(n, dtype=np.uint64) * 2048 + 14).astype(np.uint64)
            span = n * 2048
        nbytes = int(lens.astype(np.uint64).sum())
        buf = torch.empty(span + 64, dtype=torch.uint8, device=dev)
        wc.synth_fill(buf, 1, nbytes=span)
        d_off, d_len = torch.from_numpy(offs).to(dev), torch.from_numpy(lens).to(dev)
        if args.headers:
            synth.stamp_udp_headers(buf, d_off, d_len)
        out = torch.empty(n, dtype=torch.uint16, device=dev)
        run = lambda: wc.cksum_ragged(buf, d_off, d_len, out=out, kind=args.kind, check=False)  # noqa: E731
        if args.fused:
            run = lambda: wc.cksum_ip_udp_ragged(buf, d_off, d_len, check=False)  # noqa: E731
    else:
        L = 1472 if args.config == "c2" else args.len
        n = args.packets
        stride = args.stride or L
        nbytes = n * L
        # Bytes a batch pulls through the caches: its span when packed, about
        # one line pair per packet when sparse (bench.py's rotation rule).
        touched = n * min(stride, L + 128) if stride > L + 128 else args.offset + n * stride
        K = max(1, -(-args.rotate_bytes // touched)) if args.rotate_bytes else 1
        bufs = []
        for k in range(K):
            b = torch.empty(args.offset + n * stride + 64, dtype=torch.uint8, device=dev)
            wc.synth_fill(b, 1 + k)
            if args.headers:
                synth.stamp_udp_headers(b, torch.arange(n, device=dev) * stride + args.offset,
                                        torch.full((n,), L, device=dev))
            bufs.append(b)
        buf = bufs[0]
        out = torch.empty(n, dtype=torch.uint16, device=dev)
        rot = [0]

        def run():
            rot[0] = (rot[0] + 1) % K
            wc.cksum_strided(bufs[rot[0]], stride, L, n, out=out, kind=args.kind,
                             byte_offset=args.offset)
        if K > 1:
            print(f"rotating over {K} buffers", flush=True)
        if args.fused:
            run = lambda: wc.cksum_ip_udp_strided(buf, stride, L, n,  # noqa: E731
                                                  byte_offset=args.offset)
        if args.ragged:
            d_off = torch.arange(n, dtype=torch.int64, device=dev) * stride + args.offset
            d_len = torch.full((n,), L, dtype=torch.int16, device=dev)
            run = lambda: wc.cksum_ragged(buf, d_off, d_len, out=out, kind=args.kind, check=False)  # noqa: E731
            if args.fused:
                run = lambda: wc.cksum_ip_udp_ragged(buf, d_off, d_len, check=False)  # noqa: E731

    variants = [("" if v.strip() == "default" else v.strip()) for v in args.variants.split(";") if v.strip()] or [""]
    # Every WC_* knob a variant may set is reset before the next variant runs.
    knobs = {"WC_SHAPE", "WC_NT", "WC_BLOCKS_PER_CU", "WC_GRID", "WC_FLAT_UN", "WC_FLAT_TPW",
             "WC_DIAG_NOLOAD", "WC_FLAT_MIN", "WC_RAGGED_SHAPE", "WC_VARIANT", "WC_SEG",
             "WC_SEG_ROWS", "WC_GRP_DENSE", "WC_GRP_SPARSE", "WC_GRP_ROWS",
             "WC_STRIDED_SEG", "WC_FLAT_PK", "WC_GATHER", "WC_RX_EARLY", "WC_RX_HDRT", "WC_RX_SKIP",
             "WC_RX_ADAPT", "WC_RX_GRID", "WC_RX_FORCE", "WC_LEAN_PHASE", "WC_SPLIT_PKTS", "WC_SPLIT_BYTES"}
    knobs |= {kv.split("=", 1)[0] for v in variants for kv in v.split()}
    knobs |= {k for k in os.environ if k.startswith("WC_") and k != "WC_NO_BUILD"}
    base_env = {k: os.environ.get(k) for k in knobs}

    def apply(spec):
        for k, v in base_env.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        for kv in spec.split():
            k, v = kv.split("=", 1)
            os.environ[k] = v
        wc.reload_config()  # the library reads WC_* once

    cases = [(v, None) for v in variants]
    slib = None
    if args.ceiling:
        slib = stream_lib()
        sink = torch.zeros(1 << 22, dtype=torch.int32, device=dev)
        if args.config in ("zslots", "rx", "zrx"):
            # the ring's own lines, cheapest addressing (stream_ceiling.hip
            # k_slot_read): IP packets at +14 (zslots) or whole frames at +0
            # of each 2048-B slot (rx / zrx: exactly the bytes the RX
            # verdict's bandwidth is counted on)
            for grp in (8, 16):
                for grid in (16384,):
                    for nt in (1,):
                        cases.append((f"SLOTREAD G={grp} grid={grid} nt={nt}", (grp, grid, nt)))
            # exactly the 128-B lines the ring's packets / frames touch, read once
            r_off, r_len = (offs, lens) if args.config == "zslots" else (f_off, f_len)
            d_lines = torch.from_numpy(touched_lines(r_off, r_len)).to(dev)
            print(f"LINEREAD: {d_lines.numel()} lines = {d_lines.numel() * 128 / nbytes:.3f} x "
                  f"the counted bytes", flush=True)
            for u in (1, 2, 4, 8):
                cases.append((f"LINEREAD U={u}", (u, 0, 0)))
        else:
            for region in (4096, 8192, 16384, 32768, 65536):
                for mode in (0, 1):
                    for rows in (4,):
                        cases.append((f"TILEREAD region={region} mode={mode} rows={rows}",
                                      (region, mode, rows)))
            for grid in (1024, 2048, 4096, 8192):
                for unroll in (2, 4, 8):
                    for nt in (0, 1):
                        cases.append((f"READ grid={grid} unroll={unroll} nt={nt}",
                                      (grid, unroll, nt)))

    times = {c[0]: [] for c in cases}
    ref = None
    rot = locals().get("rot") if args.config in ("c2", "c3") and not (args.fused or args.ragged) else None
    for r in range(args.rounds):
        for name, cfg in cases:
            if cfg is None:
                apply(name)
                try:
                    run()  # warm + plan
                except wc.WcError as e:  # e.g. a WC_SHAPE that is not instantiated
                    print(f"!! variant {name!r} skipped: {e}", flush=True)
                    times[name].append(float("inf"))
                    continue
                t_w = time.perf_counter()
                while (time.perf_counter() - t_w) * 1e3 < args.warm_ms:
                    for _ in range(8):
                        run()
                    torch.cuda.synchronize()
                ms = time_it(run, args.iters, stream)
                if r == 0:
                    if rot is not None:  # compare every variant on the same buffer
                        rot[0] = -1
                        run()
                    res = out.cpu().numpy().copy()
                    if ref is None:
                        ref = res
                    elif not np.array_equal(ref, res):
                        print(f"!! variant {name!r} results differ", flush=True)
            else:
                g, u, nt = cfg
                rb = [0]
                pool = bufs if args.config in ("c2", "c3") else [buf]

                def fn():  # the plain read of the batch, rotating like the checksum
                    rb[0] = (rb[0] + 1) % len(pool)
                    slib.stream_read(pool[rb[0]].data_ptr(), nbytes, g, u, nt,
                                     sink.data_ptr(), stream.cuda_stream)
                if name.startswith("TILEREAD"):
                    fn = lambda: slib.tile_read(buf.data_ptr(), nbytes, g, u, nt,  # noqa: E731
                                                sink.data_ptr(), stream.cuda_stream)
                if name.startswith("LINEREAD"):
                    fn = lambda: slib.line_read(buf.data_ptr(), d_lines.data_ptr(),  # noqa: E731
                                                d_lines.numel(), g, sink.data_ptr(),
                                                stream.cuda_stream)
                if name.startswith("SLOTREAD"):
                    fn = lambda: slib.slot_read(buf.data_ptr(), 2048,  # noqa: E731
                                                14 if args.config == "zslots" else 0,
                                                d_len.data_ptr(), n, g, u, nt, sink.data_ptr(),
                                                stream.cuda_stream)
                fn()
                ms = time_it(fn, args.iters, stream)
            times[name].append(ms)
            if args.verbose:
                print(f"  round {r} {name or 'default':<40} {ms * 1e3:9.1f} us", flush=True)
    apply("")
    rows = []
    for name, ts in times.items():
        med, best = statistics.median(ts), min(ts)
        rows.append({"variant": name or "default", "ms_med": med, "ms_best": best,
                     "GBps_med": nbytes / med / 1e6, "GBps_best": nbytes / best / 1e6})
    for row in rows:
        print(f"{row['variant']:<48} {row['ms_med']*1e3:9.1f} us  "
              f"{row['GBps_med']:8.1f} GB/s med  {row['GBps_best']:8.1f} best  "
              f"{row['GBps_med']/8000*100:5.1f}% of 8 TB/s", flush=True)
    if args.json:
        Path(args.json).write_text(json.dumps({"config": args.config, "bytes": nbytes,
                                               "rows": rows}, indent=1))


if __name__ == "__main__":
    main()

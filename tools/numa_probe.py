#!/usr/bin/env python3
"""Does the host NUMA node of a batch's pages set the end-to-end rate?

    python tools/numa_probe.py [--reps 5] [--align]

Prints the GPU's NUMA node (sysfs, from its PCI bus id), this process's
allowed CPUs per node, then for each node that has allowed CPUs: C2's bytes
first-touched by this process pinned to that node's CPUs, page-locked in
place (wc_host_register) and run through wc_cksum_host (best of --reps), and
the H2D copy of the same bytes (torch copy_).  Results are checked against
the oracle.  A measurement tool, not product code.
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
os.environ.setdefault("WC_TUNING", "0")

import numpy as np  # noqa: E402
import torch  # noqa: E402

import warpcore_amd as wc  # noqa: E402
from oracle import c_oracle  # noqa: E402  (checker only)


def cpulist(text: str) -> set:
    out = set()
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--packets", type=int, default=1 << 20)
    args = ap.parse_args()
    allowed = os.sched_getaffinity(0)
    nodes = {}
    for d in sorted(Path("/sys/devices/system/node").glob("node[0-9]*")):
        cpus = cpulist((d / "cpulist").read_text()) & allowed
        nodes[int(d.name[4:])] = cpus
    props = torch.cuda.get_device_properties(0)
    try:
        bus = (f"{getattr(props, 'pci_domain_id', 0):04x}:{props.pci_bus_id:02x}:"
               f"{props.pci_device_id:02x}.0")
        gnode = int(Path(f"/sys/bus/pci/devices/{bus}/numa_node").read_text())
    except (AttributeError, OSError, ValueError):
        bus, gnode = "?", None
    print(f"GPU {bus} numa_node {gnode}; allowed CPUs per node:",
          {k: len(v) for k, v in nodes.items()}, flush=True)
    wc.gpu_init(0)
    dev = torch.device("cuda:0")
    n, L = args.packets, 1472
    d = torch.empty(n * L, dtype=torch.uint8, device=dev)
    wc.synth_fill(d, 7, nbytes=n * L)
    src = d.cpu().numpy()
    want = c_oracle.cksum_strided(src, L, L, n, kind=0)
    off = np.arange(n, dtype=np.uint64) * np.uint64(L)
    ln = np.full(n, L, dtype=np.uint16)
    for node, cpus in nodes.items():
        if not cpus:
            continue
        os.sched_setaffinity(0, cpus)
        buf = np.empty(n * L, dtype=np.uint8)  # fresh pages, first touched on `node`
        buf[:] = src
        os.sched_setaffinity(0, allowed)
        wc.host_register(buf)
        try:
            got = wc.cksum_host(buf, off, ln, kind="ip")
            bad = int((got != want).sum())
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                wc.cksum_host(buf, off, ln, kind="ip")
                ts.append(time.perf_counter() - t0)
            tc = []
            hb = torch.from_numpy(buf)
            for _ in range(args.reps):
                t0 = time.perf_counter()
                d.copy_(hb, non_blocking=True)
                torch.cuda.synchronize()
                tc.append(time.perf_counter() - t0)
        finally:
            wc.host_unregister(buf)
        print(f"pages first touched on node {node}: wc_cksum_host registered "
              f"{n * L / min(ts) / 1e9:.2f} GB/s, H2D copy {n * L / min(tc) / 1e9:.2f} GB/s, "
              f"mismatches {bad}", flush=True)


def align_probe(args) -> None:
    """The same call with the batch's start at several offsets from a page
    boundary (bench.py's batch is a torch CPU tensor, whose start is not
    page-aligned), and from a torch CPU tensor as bench.py makes it."""
    dev = torch.device("cuda:0")
    n, L = args.packets, 1472
    d = torch.empty(n * L, dtype=torch.uint8, device=dev)
    wc.synth_fill(d, 7, nbytes=n * L)
    src = d.cpu().numpy()
    want = c_oracle.cksum_strided(src, L, L, n, kind=0)
    off = np.arange(n, dtype=np.uint64) * np.uint64(L)
    ln = np.full(n, L, dtype=np.uint16)
    big = np.empty(n * L + 8192, dtype=np.uint8)
    base = (-big.ctypes.data) % 4096
    cases = [(f"page + {k}", big[base + k: base + k + n * L]) for k in (0, 16, 64, 256, 2048)]
    cases.append((f"torch CPU tensor (start mod 4096 = {src.ctypes.data % 4096})", src))
    cases.append(("the tensor again, after a torch H2D copy from it while registered", src))
    for name, buf in cases:
        if buf is not src:
            buf[:] = src
        if name.startswith("the tensor again"):
            # bench.py's e2e leg: the copy ceiling registers the batch, copies
            # it with torch, unregisters it; then the calls register it again
            wc.host_register(buf)
            d.copy_(torch.from_numpy(buf), non_blocking=True)
            torch.cuda.synchronize()
            wc.host_unregister(buf)
        wc.host_register(buf)
        try:
            bad = int((wc.cksum_host(buf, off, ln, kind="ip") != want).sum())
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                wc.cksum_host(buf, off, ln, kind="ip")
                ts.append(time.perf_counter() - t0)
        finally:
            wc.host_unregister(buf)
        print(f"{name}: wc_cksum_host registered {n * L / min(ts) / 1e9:.2f} GB/s, "
              f"mismatches {bad}", flush=True)


if __name__ == "__main__":
    if "--align" in sys.argv:
        sys.argv.remove("--align")
        _ap = argparse.ArgumentParser()
        _ap.add_argument("--reps", type=int, default=5)
        _ap.add_argument("--packets", type=int, default=1 << 20)
        wc.gpu_init(0)
        align_probe(_ap.parse_args())
        sys.exit(0)
    main()

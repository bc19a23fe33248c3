#!/usr/bin/env python3
"""Benchmark: device-resident RFC 1071 checksum of synthetic packet batches on
MI355X (BASELINE.json metric "GiB/s payload checksummed (device-resident),
1472 B pkts; % of HBM-read peak").

One step = one pass of the hot path (one wc_cksum_* launch) over one batch
that is already resident in HBM.  Default workload = BASELINE configs[1] (C2):
2^20 packets x 1472 B per GPU, stride 1472, splitmix64 bytes.  With --gpus N
(one process per GPU, torchrun) every rank checksums its own C2 batch: the
path shards by packet with no data-path collective ("scaling": "weak"); ranks
meet only at the barriers around the timed region and in the max-over-ranks
time reduction.

    python bench.py [--gpus N] [--steps K] [--warmup W]
                    [--config c2|c3|c4|c5|slots|zslots|rx|zrx] [--len L] [--kind ip|payload]
                    [--headers] [--fused] [--batches K] [--rotate-bytes B]
                    [--cpu-seconds S] [--no-cpu-baseline] [--no-c5] [--no-extra]

HBM, not the Infinity Cache: a strided batch smaller than --rotate-bytes
(1 GiB, 4x the 256 MiB Infinity Cache, MI355X_MICROARCH.md "Infinity Cache")
is run as K = ceil(1 GiB / batch) distinct batches, each with its own seed,
step i checksumming batch i mod K, so no step re-reads bytes the cache still
holds; every packet of every batch is checked.  C2's 1.54 GB batch is K = 1.

Every default line also carries (after the headline's timed region):
* "c5": SURVEY C5, the north star's strong-scaling curve -- 2^28 x 1472 B in
  total, split evenly over the N ranks, each rank's share checksummed as
  launches over a resident 2^25-packet (49 GB) window -- timed with its own
  barriers and max over ranks, with sampled parity on every rank.
* "c3": BASELINE configs[2], the MTU sweep 64/256/576/1472/9000 B x 2^20 on
  rotating batches (>= 1 GiB footprint), each size's frac from HBM plus the
  single-buffer figure as frac_l3_resident, every packet checked;
* "c4": BASELINE configs[3], 2^24 Zipf(1) 64-1472 B packets packed, every
  packet checked;
* roofline.frac_rotating: C2 over 4 rotating 1.54 GB batches.
--no-extra skips c3 / c4 / frac_rotating, --no-c5 the C5 leg.
--fused runs the fused IPv4 header + payload_cksum pass (wc_cksum_ip_udp_*).
--config rx is the RX verdict pass (wc_rx_verdict_ragged) over a netmap RX
ring of well-formed UDP frames (2048-B slots, valid IPv4 / IPv6 checksums).
--config slots is a netmap RX ring drained into one ragged batch
(backend_netmap.c:379-391): 2^20 IP packets of --len + 28 B (1500 B) in
2048-B buffers at +14 (eth.h:44-48), through wc_cksum_ragged; use it with
--kind payload --headers for the RX verify pass of udp.c:132-139.

Rank 0 prints ONE JSON line (see DESIGN.md section 6 for every field).
"""
from __future__ import annotations

import argparse
import copy
import gc
import json
import os
import sys
import time
from pathlib import Path
from types import SimpleNamespace

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "GiB/s payload checksummed (device-resident), 1472 B pkts; % of HBM-read peak"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
GIB = float(1 << 30)
C3_SIZES = (64, 256, 576, 1472, 9000)  # BASELINE configs[2]
BATCH_SEED_STEP = 0x9E3779B9  # seed of batch k = rank seed + k * this


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2",
                    choices=["c2", "c3", "c4", "c5", "slots", "zslots", "rx", "zrx"])
    ap.add_argument("--len", type=int, default=1472, help="packet bytes for c3")
    ap.add_argument("--kind", default="ip", choices=["ip", "payload"],
                    help="ip_cksum (default) or payload_cksum per packet")
    ap.add_argument("--fused", action="store_true",
                    help="fused IPv4 header checksum + payload_cksum pass (wc_cksum_ip_udp_*; "
                         "implies --kind payload --headers)")
    ap.add_argument("--no-c5", action="store_true",
                    help="skip the C5 strong-scaling leg every line carries by default")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the c3 / c4 objects and C2's frac_rotating")
    ap.add_argument("--c5-steps", type=int, default=3,
                    help="at least this many timed steps of the C5 leg (and >= 0.5 s)")
    ap.add_argument("--headers", action="store_true",
                    help="stamp well-formed IPv4 / IPv6 UDP headers on every packet "
                         "(synth.stamp_udp_headers) instead of random header bytes")
    ap.add_argument("--total-packets", type=int, default=1 << 28, help="c5 total")
    ap.add_argument("--window-packets", type=int, default=1 << 25, help="c5 resident window")
    ap.add_argument("--packets", type=int, default=1 << 20)
    ap.add_argument("--stride", type=int, default=0,
                    help="c2/c3: packet stride (default: the packet length, packed)")
    ap.add_argument("--offset", type=int, default=0,
                    help="c2/c3: byte offset of packet 0 (14: IP packets in netmap slots)")
    ap.add_argument("--batches", type=int, default=0,
                    help="c2/c3: distinct batches the steps rotate over (0: enough for "
                         "--rotate-bytes)")
    ap.add_argument("--rotate-bytes", type=int, default=1 << 30,
                    help="c2/c3: smallest footprint of the rotating batches (default 1 GiB, "
                         "4x the Infinity Cache)")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="replay the timed launches from a captured hipGraph (auto: for c3, "
                         "where a Python launch can take longer than the kernel)")
    ap.add_argument("--rx-arp", type=int, default=0,
                    help="rx / zrx: every K-th frame an ARP frame (needs no UDP check)")
    ap.add_argument("--no-rings", action="store_true",
                    help="skip the netmap RX-ring legs (rx, zrx, zrx with ARP) of the default line")
    ap.add_argument("--c3-packets", type=int, default=1 << 20, help="packets per c3 size")
    ap.add_argument("--ring-packets", type=int, default=1 << 20,
                    help="frames of the MTU ring leg (the mixed-size ring legs: twice as "
                         "many at the default)")
    ap.add_argument("--c4-packets", type=int, default=1 << 24, help="packets of the c4 object")
    ap.add_argument("--extra-seconds", type=float, default=0.25,
                    help="timed seconds per c3 / c4 / frac_rotating measurement")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="total CPU-baseline time budget (all-thread + 1-core trials)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads for the all-core CPU baseline (default: the box's share)")
    ap.add_argument("--warmup-seconds", type=float, default=1.0,
                    help="keep warming up (untimed) until this long has passed, so the "
                         "GPU clock has ramped from idle before the timed steps")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the end-to-end (host memory in and out) object")
    ap.add_argument("--e2e-packets", type=int, default=1 << 20,
                    help="packets per rank of each end-to-end call")
    ap.add_argument("--e2e-reps", type=int, default=5, help="timed calls per e2e case")
    ap.add_argument("--traffic-file", default=str(ROOT / "profiles" / "traffic.json"))
    return ap.parse_args(argv)


def resolve_launch(args, env=None):
    """How this process runs (decided before anything touches the GPU):
    ("spawn", N) -- `--gpus N > 1` without a torchrun environment: start N
    fresh ranks as children; ("rank", world) -- run as one rank of `world`.
    Raises SystemExit if a torchrun world disagrees with --gpus."""
    env = os.environ if env is None else env
    if args.gpus < 1:
        raise SystemExit(f"--gpus must be >= 1, not {args.gpus}")
    if "WORLD_SIZE" not in env:
        return ("spawn", args.gpus) if args.gpus > 1 else ("rank", 1)
    world = int(env["WORLD_SIZE"])
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: refusing to "
                         f"report a {world}-rank run as {args.gpus} GPUs")
    return "rank", world


def spawn_ranks(n, argv):
    """Run this bench as n ranks (one process per GPU) under
    torch.distributed.run and relay its exit code; rank 0's JSON line goes
    straight to our stdout.  The parent never initialises the GPU and never
    re-execs itself: the ranks are fresh child processes."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
           "--master-port", str(port), str(Path(__file__).resolve()), *argv]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def dist_setup(args):
    """One process per GPU (torchrun env).  Backend "nccl" = RCCL over xGMI;
    WC_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (tests only)."""
    _, world = resolve_launch(args)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    backend = os.environ.get("WC_DIST_BACKEND", "nccl")
    if world > 1 and backend == "nccl" and ndev < world:
        raise SystemExit(f"{world} ranks over RCCL need {world} GPUs, {ndev} visible "
                         "(WC_DIST_BACKEND=gloo rehearses ranks sharing a GPU)")
    dev_index = local % max(ndev, 1)
    torch.cuda.set_device(dev_index)
    coll_dev = torch.device("cuda", dev_index)
    # WC_DIST_FORCE_PG=1 sets up the process group even for one rank: a
    # 1-GPU box can then run bench's RCCL code path (barriers, max/sum
    # reductions, the results all-gather) end to end.
    if world > 1 or os.environ.get("WC_DIST_FORCE_PG") == "1":
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world,
                                    device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
            coll_dev = torch.device("cpu")
    return rank, dev_index, world, coll_dev


def rotation(batch_bytes: int, args) -> int:
    """Distinct batches a strided workload rotates over: --batches, else
    enough that their footprint reaches --rotate-bytes."""
    if args.batches > 0:
        return args.batches
    return max(1, -(-int(args.rotate_bytes) // max(int(batch_bytes), 1)))


def make_workload(args, dev, rank, world):
    """The workload of this run on this rank: a namespace with `step(i)` (one
    launch over batch i mod K), the packets and algorithmic bytes per step,
    `batches` (K dicts of buf / out / out_hdr), the kernel plan, description,
    config metadata, layout (`shape`) and scaling."""
    import warpcore_amd as wc
    from warpcore_amd import dist as wdist
    from warpcore_amd import synth

    seed = synth.SEED + rank
    kind = args.kind
    fused = args.fused
    if args.config == "c5":
        L = 1472
        lo, hi = wdist.shard_range(args.total_packets, rank, world)
        share = hi - lo
        win = min(share, args.window_packets)
        launches = (share + win - 1) // win
        buf = torch.empty(win * L + 64, dtype=torch.uint8, device=dev)
        wc.synth_fill(buf, seed, nbytes=win * L)
        out = torch.empty(win, dtype=torch.uint16, device=dev)
        counts = [min(win, share - k * win) for k in range(launches)]

        def step(i=0):
            for c in counts:
                wc.cksum_strided(buf, L, L, c, out=out, kind=kind)

        plan = wc.plan_strided(buf.data_ptr(), L, L, win, kind=kind)
        desc = (f"C5: {args.total_packets} x {L} B in total, rank share {share} packets as "
                f"{launches} launch(es) over a resident {win}-packet window")
        meta = {"packets_total": args.total_packets, "packets_per_gpu": share,
                "packet_bytes": L, "layout": "strided", "launches_per_step": launches,
                "kind": kind}
        return SimpleNamespace(step=step, n=share, nbytes=share * L,
                               batches=[{"buf": buf, "out": out}], plan=plan, desc=desc,
                               meta=meta, shape=(L, L, 0), scaling="strong")
    if args.config in ("rx", "zrx"):
        # netmap RX ring (backend_netmap.c:379-391): one well-formed UDP
        # frame per 2048-B slot, valid IPv4 header and UDP checksums; one
        # step = the RX verdict of every frame (wc_rx_verdict_ragged).
        slot = 2048
        if args.config == "rx":
            n = args.packets
            ip_lens = np.full(n, args.len + 28, dtype=np.uint16)
        else:
            n = 1 << 21 if args.packets == (1 << 20) else args.packets
            ip_lens = synth.zipf_lengths(n, seed=synth.ZIPF_SEED + rank)
        buf = torch.empty(n * slot + 64, dtype=torch.uint8, device=dev)
        wc.synth_fill(buf, seed, nbytes=n * slot)
        f_off, f_len = synth.make_rx_ring(buf, n, ip_lens, slot=slot)
        if args.rx_arp:  # every K-th frame ARP: its EtherType rules it out (eth.c:75-86)
            sel = torch.from_numpy(f_off[::args.rx_arp].astype(np.int64)).to(dev)
            buf[sel + 12] = 0x08
            buf[sel + 13] = 0x06
        d_off = torch.from_numpy(f_off).to(dev)
        d_len = torch.from_numpy(f_len).to(dev)
        out = torch.empty(n, dtype=torch.uint8, device=dev)
        drops = torch.zeros(1, dtype=torch.int64, device=dev)
        wc.rx_verdict_ragged(buf, d_off, d_len, out=out, drops=drops)  # validates the layout

        def step(i=0):
            wc.rx_verdict_ragged(buf, d_off, d_len, out=out, check=False, drops=drops)

        nbytes = int(f_len.astype(np.uint64).sum())
        desc = (f"netmap RX ring: {n} Ethernet frames ({'Zipf 64-1472 B IP, mean ' if args.config == 'zrx' else ''}"
                f"{nbytes / n:.1f} B) in {slot}-B slots, RX verdict (IPv4 header + UDP "
                f"checksums, ip4_rx + udp_rx checks) per frame")
        meta = {"packets_per_gpu": n, "mean_frame_bytes": round(nbytes / n, 2), "slot_bytes": slot,
                "layout": "ragged", "kind": "rx_verdict"}
        if args.rx_arp:
            meta["arp_every"] = args.rx_arp
            desc += f"; every {args.rx_arp}th frame ARP (no UDP check)"
        if args.config == "rx":
            meta["packet_bytes"] = args.len + 42  # frame: Ethernet 14 + IP/UDP 28 + payload
        plan = {"kernel": "k_rx_verdict (header parse + gathered seg stream)",
                "grid": int((n + 255) // 256)}
        return SimpleNamespace(step=step, n=n, nbytes=nbytes,
                               batches=[{"buf": buf, "out": out}], plan=plan, desc=desc,
                               meta=meta, shape=(f_off, f_len), scaling="weak")
    if args.config in ("c2", "c3"):
        L = 1472 if args.config == "c2" else args.len
        n = args.packets
        stride, at = args.stride or L, args.offset
        nbytes = n * L
        span = at + n * stride
        # bytes the steps touch: whole packets, or (sparse slots) a packet's
        # lines -- the footprint the rotation must carry past the L3
        K = rotation(n * min(stride, L + 128) if stride > L else nbytes, args)
        batches = []
        for k in range(K):
            buf = torch.empty(span + 64, dtype=torch.uint8, device=dev)
            wc.synth_fill(buf, seed + k * BATCH_SEED_STEP, nbytes=span)
            if args.headers:
                synth.stamp_udp_headers(buf, torch.arange(n, device=dev) * stride + at,
                                        torch.full((n,), L, device=dev))
            batches.append({"buf": buf, "out": torch.empty(n, dtype=torch.uint16, device=dev),
                            "out_hdr": torch.empty(n, dtype=torch.uint16, device=dev)
                            if fused else None})

        def step(i=0):
            b = batches[i % K]
            if fused:
                wc.cksum_ip_udp_strided(b["buf"], stride, L, n, out_hdr=b["out_hdr"],
                                        out=b["out"], byte_offset=at)
            else:
                wc.cksum_strided(b["buf"], stride, L, n, out=b["out"], kind=kind, byte_offset=at)

        plan = wc.plan_strided(batches[0]["buf"].data_ptr() + at, stride, L, n, kind=kind)
        desc = (f"C2: {n} x {L} B packets, stride {L}, device-resident"
                if args.config == "c2" else f"C3: {n} x {L} B packets, stride {stride}")
        if at:
            desc += f", packet 0 at +{at}"
        if K > 1:
            desc += (f"; steps rotate over {K} distinct batches ({K * span / GIB:.2f} GiB, "
                     f"past the 256 MiB Infinity Cache)")
        meta = {"packets_per_gpu": n, "packet_bytes": L, "layout": "strided", "kind": kind,
                "batches": K, "footprint_bytes": K * span}
        if stride != L or at:
            meta.update(stride=stride, offset=at)
        if fused:
            desc += ", fused IPv4 header + payload_cksum pass"
        return SimpleNamespace(step=step, n=n, nbytes=nbytes, batches=batches, plan=plan,
                               desc=desc, meta=meta, shape=(L, stride, at), scaling="weak")
    if args.config in ("slots", "zslots"):
        # netmap RX ring drained into one ragged batch: one IP packet per
        # 2048-B slot at +14 (eth.h:44-48); slots = fixed --len + 28 B,
        # zslots = C4's Zipf 64-1472 B lengths (a ring of mixed sizes)
        slot, at = 2048, 14
        if args.config == "slots":
            n = args.packets
            lens = np.full(n, args.len + 28, dtype=np.uint16)
        else:
            n = 1 << 21 if args.packets == (1 << 20) else args.packets
            lens = synth.zipf_lengths(n, seed=synth.ZIPF_SEED + rank)
        L = int(lens[0])
        offs = (np.arange(n, dtype=np.uint64) * slot + at).astype(np.uint64)
        nbytes = int(lens.astype(np.uint64).sum())
        buf = torch.empty(n * slot + 64, dtype=torch.uint8, device=dev)
        wc.synth_fill(buf, seed, nbytes=n * slot)
        d_off = torch.from_numpy(offs).to(dev)
        d_len = torch.from_numpy(lens).to(dev)
        if args.headers:
            synth.stamp_udp_headers(buf, d_off, d_len)
        out = torch.empty(n, dtype=torch.uint16, device=dev)
        out_hdr = torch.empty(n, dtype=torch.uint16, device=dev) if fused else None

        wc.cksum_ragged(buf, d_off, d_len, out=out, kind=kind)  # validates the layout once

        def step(i=0):
            if fused:
                wc.cksum_ip_udp_ragged(buf, d_off, d_len, check=False, out_hdr=out_hdr, out=out)
            else:
                wc.cksum_ragged(buf, d_off, d_len, out=out, kind=kind, check=False)

        if args.config == "slots":
            desc = (f"netmap RX ring: {n} x {L} B IP packets in {slot}-B slots at +{at}, "
                    f"ragged batch")
            meta = {"packets_per_gpu": n, "packet_bytes": L, "slot_bytes": slot,
                    "layout": "ragged", "kind": kind}
        else:
            desc = (f"netmap RX ring of mixed sizes: {n} Zipf(s=1) 64-1472 B packets "
                    f"(mean {nbytes / n:.1f}) in {slot}-B slots at +{at}, ragged batch")
            meta = {"packets_per_gpu": n, "mean_packet_bytes": round(nbytes / n, 2),
                    "slot_bytes": slot, "layout": "ragged", "kind": kind}
        if fused:
            desc += ", fused IPv4 header + payload_cksum pass"
        path = "grouped path" if args.config == "slots" and not fused else "gathered-stream path"
        plan = {"kernel": f"seg ({path} for these tiles)",
                "rows_per_group": int(os.environ.get(
                    "WC_GRP_ROWS" if args.config == "slots" else "WC_SEG_ROWS", "4")),
                "grid": int((n + 255) // 256)}
        return SimpleNamespace(step=step, n=n, nbytes=nbytes,
                               batches=[{"buf": buf, "out": out, "out_hdr": out_hdr}],
                               plan=plan, desc=desc, meta=meta, shape=(offs, lens),
                               scaling="weak")
    # C4: Zipf(1) lengths 64..1472 B, packed with no padding (unaligned starts)
    n = 1 << 24 if args.packets == (1 << 20) else args.packets
    lens = synth.zipf_lengths(n, seed=synth.ZIPF_SEED + rank)
    offs = synth.packed_offsets(lens)
    nbytes = int(lens.astype(np.uint64).sum())
    buf = torch.empty(nbytes + 64, dtype=torch.uint8, device=dev)
    wc.synth_fill(buf, seed, nbytes=nbytes)
    d_off = torch.from_numpy(offs).to(dev)
    d_len = torch.from_numpy(lens).to(dev)
    if args.headers:
        synth.stamp_udp_headers(buf, d_off, d_len)
    out = torch.empty(n, dtype=torch.uint16, device=dev)
    out_hdr = torch.empty(n, dtype=torch.uint16, device=dev) if fused else None

    wc.cksum_ragged(buf, d_off, d_len, out=out, kind=kind)  # validates the layout once

    def step(i=0):
        if fused:
            wc.cksum_ip_udp_ragged(buf, d_off, d_len, check=False, out_hdr=out_hdr, out=out)
        else:
            wc.cksum_ragged(buf, d_off, d_len, out=out, kind=kind, check=False)

    desc = f"C4: {n} packets, Zipf(s=1) lengths 64-1472 B (mean {nbytes / n:.1f}), packed"
    meta = {"packets_per_gpu": n, "mean_packet_bytes": round(nbytes / n, 2),
            "layout": "ragged", "kind": kind}
    if fused:
        desc += ", fused IPv4 header + payload_cksum pass"
    seg = int(os.environ.get("WC_SEG", "1"))
    if seg != 0:
        plan = {"kernel": "seg (segmented prefix over dense 64-packet tiles, flat fallback)",
                "rows_per_group": int(os.environ.get("WC_SEG_ROWS", "4")),
                "grid": int((n + 255) // 256)}
    else:
        plan = {"kernel": "flat (chunk-balanced, 64-packet tiles)",
                "rows_per_group": int(os.environ.get("WC_FLAT_UN", "2")),
                "grid": int((n + 255) // 256)}
    return SimpleNamespace(step=step, n=n, nbytes=nbytes,
                           batches=[{"buf": buf, "out": out, "out_hdr": out_hdr}],
                           plan=plan, desc=desc, meta=meta, shape=(offs, lens), scaling="weak")


class Timer:
    """The timed launches of one workload on torch's current stream (the
    stream every wc_* launch goes to), as plain launches or replayed from one
    captured hipGraph of `per_graph` consecutive steps (a whole number of
    rotations) -- the graph takes the Python launch cost out of small-batch
    timings (a 64-B C3 kernel is ~9 us, a Python launch about as long)."""

    def __init__(self, W, dev, use_graph: bool, rotate: int = 1, min_graph_steps: int = 8,
                 exact_steps: int = 0):
        self.W, self.dev = W, dev
        self.graph = None
        self.per_graph = 1
        if use_graph:
            K = max(1, rotate)
            # exact_steps: the graph holds exactly that many steps (the
            # headline's K timed launches, one replay); else a whole number
            # of rotations of at least min_graph_steps
            self.per_graph = exact_steps or K * max(1, -(-min_graph_steps // K))
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for i in range(self.per_graph):
                    W.step(i)
            torch.cuda.synchronize(dev)
            self.graph = g

    def rounded(self, steps: int) -> int:
        """Steps actually timed: a whole number of graph replays."""
        return max(1, -(-steps // self.per_graph)) * self.per_graph

    def run(self, steps: int, start: int = 0) -> None:
        if self.graph is not None:
            for _ in range(self.rounded(steps) // self.per_graph):
                self.graph.replay()
        else:
            for i in range(steps):
                self.W.step(start + i)

    def warm(self, steps: int, seconds: float) -> None:
        t_w = time.perf_counter()
        done = 0
        while done < steps or time.perf_counter() - t_w < seconds:
            self.run(self.per_graph, done)
            done += self.per_graph
            if done % 16 < self.per_graph:
                torch.cuda.synchronize(self.dev)
        torch.cuda.synchronize(self.dev)

    def kernel_ms(self, steps: int) -> float:
        """Average launch duration over `steps` (HIP events on the launch
        stream, one bracket around all of them)."""
        steps = self.rounded(steps)
        stream = torch.cuda.current_stream(self.dev)
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        self.run(steps)
        ev1.record(stream)
        ev1.synchronize()
        return ev0.elapsed_time(ev1) / steps

    def steps_for(self, seconds: float) -> int:
        """Steps that take about `seconds` (from one short calibration)."""
        ms = self.kernel_ms(self.per_graph)
        return self.rounded(max(self.per_graph, int(seconds * 1e3 / max(ms, 1e-3))))


def cpu_threads(args):
    """Host threads for the all-core CPU baseline: --cpu-threads, else the
    box's CPU share (OMP_NUM_THREADS, which the GPU box sets to its per-GPU
    share), else every core this process may run on."""
    try:
        visible = len(os.sched_getaffinity(0))
    except AttributeError:
        visible = os.cpu_count() or 1
    if args.cpu_threads > 0:
        return args.cpu_threads, visible, "--cpu-threads"
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and 0 < int(share) < visible:
        return int(share), visible, "OMP_NUM_THREADS (the box's CPU share)"
    return visible, visible, "sched_getaffinity"


def cpu_baseline(args, buf, shape, nbytes_total):
    """The oracle's C restatement (reference Release flags -Ofast
    -march=native, one call per packet) timed on this host's cores on a
    bounded sample: all threads and 1 core, best of 5 trials each
    (BASELINE.md section 3)."""
    from oracle import c_oracle  # checker / baseline only

    threads, visible, why = cpu_threads(args)
    k = 1 if args.kind == "payload" else 0
    trials = 5
    per_trial = max(args.cpu_seconds / (2 * trials), 0.05)
    if args.config in ("c2", "c3", "c5"):
        L, stride, at = shape
        # The whole batch (DRAM-resident on the host, far beyond its L3).
        n_s = max(1, min(args.packets, (2 << 30) // max(L, 1)))
        sample = buf[at: at + n_s * stride].cpu().numpy()

        def trial(th):
            bps, passes = c_oracle.bench_strided(sample, stride, L, n_s, kind=k, threads=th,
                                                 min_seconds=per_trial)
            return bps, passes
        desc = f"{n_s} packets x {L} B ({n_s * L / 1e9:.2f} GB, the full batch)"
    else:
        offs, lens = shape
        n_s = min(offs.size, 1 << 22 if args.config not in ("rx", "zrx") else 1 << 20)
        end = int(offs[n_s - 1]) + max(int(lens[n_s - 1]), 40)
        sample = buf[:end].cpu().numpy()
        o_s, l_s = offs[:n_s], lens[:n_s]
        sbytes = float(l_s.astype(np.uint64).sum())
        rx = args.config in ("rx", "zrx")

        def trial(th):
            t0 = time.perf_counter()
            passes = 0
            while True:
                if rx:
                    c_oracle.rx_verdict_ragged(sample, o_s, l_s, threads=th)
                else:
                    c_oracle.cksum_ragged(sample, o_s, l_s, kind=k, threads=th)
                passes += 1
                dt = time.perf_counter() - t0
                if dt >= per_trial:
                    return passes * sbytes / dt, passes
        what = "frames, oracle_rx_verdict" if rx else "packets"
        desc = (f"first {n_s} {'Zipf ' if args.config in ('c4', 'zslots', 'zrx') else ''}{what} "
                f"({end / 1e6:.0f} MB)")
    best_all = max(trial(threads)[0] for _ in range(trials))
    best_one = max(trial(1)[0] for _ in range(trials))
    try:
        model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo")
                     if l.startswith("model name"))
    except (OSError, StopIteration):
        model = "unknown"
    if args.fused:
        desc += " (payload_cksum only: the CPU port's header checksum is not timed)"
    return {"value": round(best_all / GIB, 3), "unit": "GiB/s", "cores": threads,
            "kind": "port", "value_1core": round(best_one / GIB, 3), "best_of": trials,
            "cores_visible": visible,
            "sample": f"{desc}, >= {per_trial:.2f} s per trial; oracle/wc_oracle.c -Ofast "
                      f"-march=native (reference Release flags), one call per packet, "
                      f"{threads} pthreads ({why}; {visible} cores visible) and 1 core, "
                      f"best of {trials} each, on {model}"}


def last_count(args):
    from warpcore_amd import dist as wdist
    rank, world = wdist.world()
    lo, hi = wdist.shard_range(args.total_packets, rank, world)
    share = hi - lo
    win = min(share, args.window_packets)
    return share - (share - 1) // win * win


def parity_batch(args, b, shape):
    """Bit-exact check of one batch's last results over EVERY packet against
    the oracle (run outside the timed region): (checked, mismatches, extra)."""
    from oracle import c_oracle
    buf, out, out_hdr = b["buf"], b["out"], b.get("out_hdr")
    k = 1 if args.kind == "payload" else 0
    if args.config in ("rx", "zrx"):
        offs, flens = shape
        hb = buf[: int(offs[-1]) + int(flens[-1])].cpu().numpy()
        want = c_oracle.rx_verdict_ragged(hb, offs, flens)
        got = out.cpu().numpy()
        return int(got.size), int((got != want).sum()), {
            "verdicts_ok": int(np.isin(want, (0, 1)).sum())}
    got = out.cpu().numpy().view(np.uint16)
    if args.config in ("c2", "c3", "c5"):
        hb = buf[: shape[2] + got.size * shape[1]].cpu().numpy()
    else:  # ragged: every byte up to the last packet's end (+ its header fields)
        offs, lens = shape
        hb = buf[: min(buf.numel(), int(offs[-1]) + max(int(lens[-1]), 40))].cpu().numpy()
    if args.config in ("c2", "c3", "c5"):
        # c5: the last launch of the step covered the window's first
        # `counts[-1]` packets; check the whole window result of that launch
        L, stride, at = shape
        n_chk = got.size if args.config != "c5" else min(got.size, last_count(args))
        want = c_oracle.cksum_strided(hb, stride, L, n_chk, kind=k, byte_offset=at)
        got = got[:n_chk]
        offs = np.arange(n_chk, dtype=np.uint64) * np.uint64(stride) + np.uint64(at)
    else:
        offs, lens = shape
        want = c_oracle.cksum_ragged(hb, offs, lens, kind=k)
    bad = int((got != want).sum())
    if out_hdr is not None:
        # fused pass: the IPv4 header checksums too (ip_cksum(ip, hl), 0 for IPv6)
        b0 = hb[offs.astype(np.int64)]
        v4 = (b0 >> 4) == 4
        hl = np.where(v4, (b0 & 0x0F).astype(np.uint16) * 4, 0).astype(np.uint16)
        want_h = np.where(v4, c_oracle.cksum_ragged(hb, offs, hl, kind=0), 0).astype(np.uint16)
        got_h = out_hdr.cpu().numpy().view(np.uint16)[: got.size]
        bad += int((got_h != want_h).sum())
    return int(got.size), bad, {}


def parity_check(args, W):
    """Every packet of every batch of W against the oracle."""
    checked = bad = 0
    extra = {}
    for b in W.batches:
        c, m, e = parity_batch(args, b, W.shape)
        checked += c
        bad += m
        for key, v in e.items():
            extra[key] = extra.get(key, 0) + v
    return {"checked_packets": checked, "mismatches": bad, **extra}


def c5_leg(args, dev, rank, world, coll_dev):
    """SURVEY C5 beside the headline (the north star's 1/2/4/8-GPU curve):
    2^28 x 1472 B in total, split evenly over the ranks (wc_shard_range's
    split), each rank's share checksummed as launches over a resident
    2^25-packet (49 GB) window of synthetic bytes.  Timed like the headline
    (barrier + synchronize on both sides, max over ranks); parity on three
    sampled 2^16-packet stretches of every rank's window."""
    import warpcore_amd as wc
    from oracle import c_oracle
    from warpcore_amd import dist as wdist
    from warpcore_amd import synth

    L = 1472
    lo, hi = wdist.shard_range(args.total_packets, rank, world)
    share = hi - lo
    win = min(share, args.window_packets)
    launches = (share + win - 1) // win
    counts = [min(win, share - k * win) for k in range(launches)]
    buf = torch.empty(win * L + 64, dtype=torch.uint8, device=dev)
    wc.synth_fill(buf, synth.SEED + 1000 + rank, nbytes=win * L)
    out = torch.empty(win, dtype=torch.uint16, device=dev)

    def step():
        for c in counts:
            wc.cksum_strided(buf, L, L, c, out=out, kind="ip")

    # Warm up for >= 0.3 s (the clock ramps; a fresh 49-GB window's first
    # pass), then time at least --c5-steps steps and >= 0.5 s of them (one
    # step is 55 ms at N = 1 but 7 ms at N = 8).
    t_w = time.perf_counter()
    warm = 0
    while warm < 1 or time.perf_counter() - t_w < 0.3:
        step()
        torch.cuda.synchronize(dev)
        warm += 1
    step_s = (time.perf_counter() - t_w) / warm
    steps = int(wdist.max_over_ranks(float(max(args.c5_steps, -(-0.5 // step_s))), coll_dev))
    wdist.barrier(dev)
    stream = torch.cuda.current_stream(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0  # (as the headline: to this rank's synchronize)
    wdist.barrier(dev)
    elapsed = wdist.max_over_ranks(elapsed, coll_dev)
    kernel_ms = wdist.max_over_ranks(ev0.elapsed_time(ev1) / steps / launches, coll_dev)
    total_bytes = float(args.total_packets) * L * steps
    gbps = total_bytes / elapsed / 1e9
    # sampled parity: every launch rewrote out[:count] from the same window
    m = min(1 << 16, counts[-1])
    bad = 0
    for s0 in sorted({0, (counts[-1] - m) // 2, counts[-1] - m}):
        hb = buf[s0 * L:(s0 + m) * L].cpu().numpy()
        want = c_oracle.cksum_strided(hb, L, L, m, kind=0)
        bad += int((out[s0:s0 + m].cpu().numpy().view(np.uint16) != want).sum())
    checked = wdist.sum_over_ranks(3 * m, coll_dev)
    bad = wdist.sum_over_ranks(bad, coll_dev)
    del buf, out
    torch.cuda.empty_cache()
    return {
        "workload": (f"SURVEY C5: {args.total_packets} x {L} B = "
                     f"{args.total_packets * L / 1e9:.1f} GB in total, split evenly over "
                     f"{world} rank(s): {share} packets per rank as {launches} launch(es) over "
                     f"a resident {win}-packet window"),
        "scaling": "strong", "n_gpus": world, "steps": steps, "warmup_steps": warm,
        "ms_per_step": round(elapsed / steps * 1e3, 3),
        "value": round(total_bytes / elapsed / GIB, 2), "unit": "GiB/s",
        "GBps": round(gbps, 1),
        "frac_job": round(gbps / (world * HBM_PEAK_GBPS), 4),
        "kernel_ms_avg_max_rank": round(kernel_ms, 4),
        "frac_kernel": round(counts[0] * L / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
        "parity": {"checked_packets": checked, "mismatches": bad,
                   "sample": "3 x 2^16 packets per rank (start, middle, end of the window)"},
    }


def _host_ring(dev, n, ip_len, seed, slot=2048):
    """A netmap ring of n well-formed UDP frames (2:1 IPv4 / IPv6, valid
    header and UDP checksums; synth.make_rx_ring) of `ip_len`-byte IP packets
    in `slot`-byte buffers, built on the device and copied to host memory
    twice: as the RX ring (checksums stored) and as the TX queue (both
    checksum fields 0, as mk_ip4_hdr / udp_tx leave them before the
    checksums are computed, ip4.c:184-186, udp.c:209-213).
    Returns (rx bytes, tx bytes, frame offsets, frame lengths)."""
    import warpcore_amd as wc
    from warpcore_amd import synth
    d = torch.empty(n * slot + 64, dtype=torch.uint8, device=dev)
    wc.synth_fill(d, seed, nbytes=n * slot)
    f_off, f_len = synth.make_rx_ring(d, n, np.full(n, ip_len, dtype=np.uint16), slot=slot)
    rx = d.cpu().numpy()
    ip = torch.from_numpy(f_off.astype(np.int64)).to(dev) + 14
    v6 = (torch.arange(n, device=dev) % 3) == 0  # make_rx_ring's v6_every
    for at4, at6 in ((10, None), (11, None), (26, 46), (27, 47)):
        d[ip[~v6] + at4] = 0
        if at6 is not None:
            d[ip[v6] + at6] = 0
    tx = d.cpu().numpy()
    del d, ip, v6
    return rx, tx, f_off, f_len


def e2e_leg(args, dev, rank, world, coll_dev):
    """North star: "this path starts and ends in host memory (netmap rings or
    socket buffers), so the end-to-end rate including pinned hipMemcpyAsync in
    and out must also be measured".  The three host-memory calls the hooks
    make, each over 2^20 packets of C2's 1472 B, in
    a registered (page-locked: wc_host_register, netmap's w->mem) and in a
    pageable host region:
      * wc_cksum_host        -- C2's strided bytes, ip_cksum;
      * wc_cksum_ip_udp_host -- the TX batch point (backend_netmap.c:348-358):
                                well-formed IPv4 / IPv6 UDP packets at +14 of
                                2048-B slots, both checksum fields 0;
      * wc_rx_verdict_host   -- the RX batch point (backend_netmap.c:379-391):
                                the same frames as a ring, checksums stored.
    Every call is timed from host memory in to host results out (one
    synchronous call: pipelined H2D, kernel, D2H), beside the measured
    hipMemcpy H2D ceiling of the same bytes (torch copy_ from pinned and from
    pageable memory).  Every result is checked against the oracle.  At N > 1
    every rank runs its own batch over its own link at the same time (barrier
    before each timed call), so GBps is the whole node's rate: N x bytes over
    the slowest rank's time."""
    import warpcore_amd as wc
    from oracle import c_oracle  # checker only
    from warpcore_amd import dist as wdist
    from warpcore_amd import synth

    n, L, reps = args.e2e_packets, 1472, max(1, args.e2e_reps)
    seed = synth.SEED + 0xE2E + rank
    d = torch.empty(n * L + 64, dtype=torch.uint8, device=dev)
    wc.synth_fill(d, seed, nbytes=n * L)
    c2 = d[: n * L].cpu().numpy()
    rx, tx, f_off, f_len = _host_ring(dev, n, L, seed + 1)
    ip_off = f_off + np.uint64(14)
    ip_len = (f_len.astype(np.int64) - 14).astype(np.uint16)

    def timed(fn):
        """best and median seconds of `reps` calls, each bracketed by a
        barrier; the slowest rank's."""
        ts = []
        for _ in range(reps):
            wdist.barrier(dev)
            t0 = time.perf_counter()
            fn()
            ts.append(wdist.max_over_ranks(time.perf_counter() - t0, coll_dev))
        return min(ts), sorted(ts)[len(ts) // 2]

    # the copy ceiling: the same C2 bytes host -> device (hipMemcpyAsync)
    pinned = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
    pinned.copy_(torch.from_numpy(c2))
    pageable = torch.from_numpy(c2)
    ceiling = {}
    for name, src in (("pinned", pinned), ("registered", pageable), ("pageable", pageable)):
        # pinned: torch's page-locked allocation (hipHostMalloc); registered:
        # the same numpy bytes page-locked in place (wc_host_register, as a
        # netmap region would be); pageable: plain memory
        def copy(src=src):
            d[: n * L].copy_(src, non_blocking=True)
            torch.cuda.synchronize(dev)
        if name == "registered":
            wc.host_register(c2)
        try:
            copy()
            best, _ = timed(copy)
        finally:
            if name == "registered":
                wc.host_unregister(c2)
        ceiling[name] = round(world * n * L / best / 1e9, 2)
    del pinned, pageable, d
    torch.cuda.empty_cache()

    # every call's expected results (oracle on the same host bytes)
    c2_off = np.arange(n, dtype=np.uint64) * np.uint64(L)
    c2_len = np.full(n, L, dtype=np.uint16)
    want_c2 = c_oracle.cksum_strided(c2, L, L, n, kind=0)
    want_pay = c_oracle.cksum_ragged(tx, ip_off, ip_len, kind=1)
    b0 = tx[ip_off.astype(np.int64)]
    v4 = (b0 >> 4) == 4
    hl = np.where(v4, (b0 & 0x0F).astype(np.uint16) * 4, 0).astype(np.uint16)
    want_hdr = np.where(v4, c_oracle.cksum_ragged(tx, ip_off, hl, kind=0), 0).astype(np.uint16)
    want_rx = c_oracle.rx_verdict_ragged(rx, f_off, f_len)

    calls = {
        "cksum_host": (c2, lambda: wc.cksum_host(c2, c2_off, c2_len, kind="ip"),
                       lambda got: int((got != want_c2).sum()), n * L),
        "cksum_ip_udp_host": (tx, lambda: wc.cksum_ip_udp_host(tx, ip_off, ip_len),
                              lambda got: int((got[0] != want_hdr).sum() +
                                              (got[1] != want_pay).sum()),
                              int(ip_len.astype(np.uint64).sum())),
        "rx_verdict_host": (rx, lambda: wc.rx_verdict_host(rx, f_off, f_len),
                            lambda got: int((got[0] != want_rx).sum()),
                            int(f_len.astype(np.uint64).sum())),
    }
    res = {}
    for name, (region, fn, bad_of, nbytes) in calls.items():
        res[name] = {"bytes_per_rank": nbytes}
        for kind in ("registered", "pageable"):
            if kind == "registered":
                wc.host_register(region)
            try:
                bad = bad_of(fn())  # warm-up call, checked
                best, med = timed(fn)
                bad += bad_of(fn())  # and the results of a timed-state call
            finally:
                if kind == "registered":
                    wc.host_unregister(region)
            gbps = world * nbytes / best / 1e9
            res[name][kind] = {
                "GBps": round(gbps, 2), "GBps_median": round(world * nbytes / med / 1e9, 2),
                "ms_best": round(best * 1e3, 3),
                "frac_of_h2d_pinned": round(gbps / ceiling["pinned"], 4),
                "frac_of_h2d_same_memory": round(gbps / ceiling[kind], 4),
                "parity": {"checked_packets": wdist.sum_over_ranks(2 * n, coll_dev),
                           "mismatches": wdist.sum_over_ranks(bad, coll_dev)}}
    rx_ok = int(np.isin(want_rx, (0, 1)).sum())
    return {
        "workload": (f"{n} packets x {L} B per rank from host memory to host results, one "
                     f"synchronous call each (pipelined hipMemcpyAsync H2D, kernel, D2H of the "
                     f"results): wc_cksum_host over C2's strided bytes; wc_cksum_ip_udp_host "
                     f"(TX) and wc_rx_verdict_host (RX) over the same {L}-B UDP/IP packets "
                     f"(2:1 IPv4/IPv6) in 2048-B netmap slots ({L + 14}-B frames); registered "
                     f"(page-locked) and pageable regions; {world} rank(s) at once, each over "
                     f"its own link; best of {reps}"),
        "n_ranks": world,
        "h2d_ceiling_GBps": {**ceiling, "how": "torch copy_ of the C2 bytes to the device "
                                              "(hipMemcpyAsync H2D) from a hipHostMalloc'd "
                                              "buffer, from the region page-locked in place, "
                                              "and from pageable memory; best of %d" % reps},
        "calls": res,
        "rx_frames_ok": wdist.sum_over_ranks(rx_ok, coll_dev),
    }


def traffic_entry(args, meta, path):
    """HBM bytes per launch for this workload from profiles/traffic.json
    (PMC FETCH_SIZE x2 + WRITE_SIZE, separate rocprofv3 passes): (bytes,
    source) or (None, None)."""
    try:
        tf = json.loads(Path(path).read_text())
    except (OSError, ValueError):
        return None, None
    key = f"{args.config}:{meta.get('packet_bytes', 'zipf')}"
    if "stride" in meta:
        key += f":s{meta['stride']}+{meta['offset']}"
    if args.kind != "ip" and args.config not in ("rx", "zrx"):
        key += f":{args.kind}"
    if args.headers and args.config not in ("rx", "zrx"):
        key += ":headers"
    if args.fused:
        key += ":fused"
    if key not in tf:
        return None, None
    e = tf[key]
    return e["hbm_bytes_per_launch"], (
        f"{os.path.relpath(path, ROOT)} [{key}] ({e.get('round', 'r01')}: rocprofv3 --pmc "
        f"FETCH_SIZE x2 + WRITE_SIZE, separate passes; a static lookup, not this run)")


_PROBES = {}


def _mhz(v: float):
    return None if v != v else round(v)  # (NaN: no two samples inside the window)


def sclk_probe(dev):
    """One shader-clock probe per device (warpcore_amd.SclkProbe)."""
    import warpcore_amd as wc
    if dev not in _PROBES:
        _PROBES[dev] = wc.SclkProbe(dev)
    return _PROBES[dev]


def measure_leg(args, dev, rank, world, coll_dev, sub, use_graph):
    """One secondary measurement (c3 size, c4, C2 rotating): build the
    workload `sub` (args with its config), warm it, time it on HIP events,
    check every packet of every batch; frees its buffers.  At K > 1 rotating
    batches it also times batch 0 alone (frac_l3_resident)."""
    from warpcore_amd import dist as wdist
    W = make_workload(sub, dev, rank, world)
    K = len(W.batches)
    T = Timer(W, dev, use_graph, rotate=K)
    T.warm(2 * T.per_graph, 0.2)
    steps = T.steps_for(args.extra_seconds)
    wdist.barrier(dev)
    # the shader clock beside the timed launches (a one-wave probe on its own
    # stream): clock-sensitive legs (the mixed-size RX ring) move with DVFS
    probe = sclk_probe(dev)
    probe.start(0.9 * args.extra_seconds * 1e3)
    ms = wdist.max_over_ranks(T.kernel_ms(steps), coll_dev)
    res = {"kernel_ms_avg_max_rank": round(ms, 5),
           "GBps": round(W.nbytes / (ms * 1e-3) / 1e9, 1),
           "frac": round(W.nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
           "batches": K, "footprint_GB": round(K * W.nbytes / 1e9, 3),
           "steps": steps, "launch": "hipGraph replay" if T.graph is not None else "stream",
           "sclk_MHz": _mhz(probe.mhz())}
    par = parity_check(sub, W)  # every batch's results are from its last timed launch
    res["parity"] = {"checked_packets": wdist.sum_over_ranks(par["checked_packets"], coll_dev),
                     "mismatches": wdist.sum_over_ranks(par["mismatches"], coll_dev)}
    if K > 1:
        one = SimpleNamespace(**vars(W))
        one.batches = W.batches[:1]
        T1 = Timer(one, dev, use_graph, rotate=1)
        T1.warm(T1.per_graph, 0.05)
        wdist.barrier(dev)
        ms1 = wdist.max_over_ranks(T1.kernel_ms(T1.steps_for(args.extra_seconds)), coll_dev)
        res["frac_l3_resident"] = round(W.nbytes / (ms1 * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
        res["kernel_ms_l3_resident"] = round(ms1, 5)
        del T1, one
    tb, _ = traffic_entry(sub, W.meta, args.traffic_file)
    res["traffic_over_algorithmic"] = round(tb / W.nbytes, 4) if tb else None
    res["kernel"] = W.plan.get("kernel")
    del T, W
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    return res


def extra_legs(args, dev, rank, world, coll_dev):
    """The default line's secondary configs, each timed on the device like
    the headline (after it): C2 over 4 rotating batches, BASELINE configs[2]
    (c3) on rotating batches and configs[3] (c4)."""
    base = copy.copy(args)
    base.kind, base.headers, base.fused, base.batches = "ip", False, False, 0
    rot = copy.copy(base)
    rot.config, rot.packets, rot.batches = "c2", args.packets, 4
    c2rot = measure_leg(args, dev, rank, world, coll_dev, rot, use_graph=False)
    c3 = {"workload": (f"BASELINE configs[2]: {args.c3_packets} packets x each size, stride = "
                       f"size, ip_cksum; steps rotate over K = ceil({args.rotate_bytes} B / "
                       f"batch) distinct seeded batches (HBM rate: frac); the single batch "
                       f"re-read (frac_l3_resident) where K > 1"),
          "sizes": {}}
    for L in C3_SIZES:
        sub = copy.copy(base)
        sub.config, sub.len, sub.packets = "c3", L, args.c3_packets
        c3["sizes"][str(L)] = measure_leg(args, dev, rank, world, coll_dev, sub, use_graph=True)
    sub = copy.copy(base)
    sub.config, sub.packets = "c4", args.c4_packets
    c4 = measure_leg(args, dev, rank, world, coll_dev, sub, use_graph=True)
    c4["workload"] = (f"BASELINE configs[3]: {args.c4_packets} packets, Zipf(s=1) lengths "
                      f"64-1472 B, packed (unaligned starts), ip_cksum")
    rings = None
    if not args.no_rings:
        # the RX verdict over netmap RX rings (device-resident),
        # beside the headline: MTU frames, C4's Zipf sizes, and the Zipf ring
        # with every third frame ARP (the default ADAPT mode's other case)
        rings = {"workload": ("netmap RX rings, one frame per 2048-B slot, the RX verdict "
                              "(wc_rx_verdict_ragged) of every frame; bytes = frame bytes; "
                              "every verdict checked against oracle_rx_verdict")}
        for name, cfg, arp in (("rx_mtu", "rx", 0), ("zrx", "zrx", 0), ("zrx_arp3", "zrx", 3)):
            sub = copy.copy(base)
            sub.config, sub.packets, sub.len, sub.rx_arp = cfg, args.ring_packets, 1472, arp
            rings[name] = measure_leg(args, dev, rank, world, coll_dev, sub, use_graph=False)
    return c2rot, c3, c4, rings


def main():
    args = parse()
    how, n_ranks = resolve_launch(args)
    if how == "spawn":
        return spawn_ranks(n_ranks, sys.argv[1:])
    from warpcore_amd import dist as wdist
    rank, local, world, coll_dev = dist_setup(args)
    dev = torch.device("cuda", local)
    import warpcore_amd as wc
    wc.gpu_init(local)
    if args.fused:  # the fused pass is payload_cksum over real UDP headers
        args.kind, args.headers = "payload", True

    W = make_workload(args, dev, rank, world)
    n, nbytes, meta = W.n, W.nbytes, W.meta
    K = len(W.batches)
    # The timed launches replay from a hipGraph for c2 (all K timed steps
    # captured once: one replay, no Python launch cost between t0 and the
    # first kernel -- VERDICT r05 item 4, tools/diag_headline.py) and c3 (a
    # whole number of rotations per graph: a 64-B batch's kernel is ~9 us).
    # (c2 over K > 1 rotating batches -- a reduced --packets -- keeps stream
    # launches: a graph of exactly K' < K steps would leave batches its
    # replays never launch, and every batch's results are checked)
    c2_graph = args.config == "c2" and K == 1
    use_graph = args.graph == "on" or (args.graph == "auto" and (args.config == "c3" or c2_graph))
    T = Timer(W, dev, use_graph, rotate=K, exact_steps=args.steps if c2_graph else 0)
    T.warm(args.warmup, args.warmup_seconds)
    wdist.barrier(dev)

    steps = T.rounded(args.steps)
    stream = torch.cuda.current_stream(dev)  # the stream every launch goes to
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    # Every rank leaves the barrier together (t0), times its own K steps until
    # its device has finished them (synchronize), and the slowest rank's time
    # is the job's (max over ranks); the closing barrier aligns the ranks
    # again outside the timed region, so its collective's own latency is not
    # counted as checksum time.
    gc.disable()  # (no collector pass inside the timed region)
    t0 = time.perf_counter()
    ev0.record(stream)
    T.run(steps)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    gc.enable()
    wdist.barrier(dev)
    kernel_ms = ev0.elapsed_time(ev1) / steps
    timing = ((f"hipGraph replay ({T.per_graph} launches per graph)" if use_graph
               else "stream launches")
              + "; whole-job time: from a barrier + synchronize to this rank's "
                "synchronize, max over ranks; kernel time from HIP events on the launch "
                "stream")

    elapsed = wdist.max_over_ranks(elapsed, coll_dev)
    kernel_ms_max = wdist.max_over_ranks(kernel_ms, coll_dev)
    total_bytes = float(wdist.sum_over_ranks(int(nbytes), coll_dev)) * steps
    value = total_bytes / elapsed / GIB
    # Roofline of the dominant kernel: one rank's algorithmic bytes per launch
    # over the slowest rank's average launch time (all ranks move the same
    # bytes); frac_job is the whole job's rate against N x peak.
    achieved = nbytes / (kernel_ms_max * 1e-3) / 1e9
    frac_job = value * GIB / 1e9 / (world * HBM_PEAK_GBPS)

    # Single-buffer figure beside a rotating run (the Infinity-Cache-resident
    # rate the rotation avoids).
    frac_l3 = None
    if K > 1:
        one = SimpleNamespace(**vars(W))
        one.batches = W.batches[:1]
        T1 = Timer(one, dev, use_graph, rotate=1)
        T1.warm(T1.per_graph, 0.1)
        wdist.barrier(dev)
        ms1 = wdist.max_over_ranks(T1.kernel_ms(steps), coll_dev)
        frac_l3 = round(nbytes / (ms1 * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
        del T1, one

    parity = parity_check(args, W)
    for key in list(parity):
        if isinstance(parity[key], int):
            parity[key] = wdist.sum_over_ranks(parity[key], coll_dev)

    # after the timed region the ranks exchange their 2-byte
    # results (RCCL all-gather over xGMI; host tensors for the gloo
    # rehearsal), so every rank holds the whole job's results in packet order.
    out = W.batches[0]["out"]
    gather = None
    if (world > 1 or wdist._pg_active()) and out.numel() == n and out.element_size() == 2:
        src = out.view(torch.int16)
        if coll_dev.type != "cuda":
            src = src.cpu()
        wdist.barrier(dev)
        t_g = time.perf_counter()
        allr = wdist.gather_results(src, world * n)
        if coll_dev.type == "cuda":
            torch.cuda.synchronize(dev)
        g_ms = (time.perf_counter() - t_g) * 1e3
        lo, hi = wdist.shard_range(world * n, rank, world)
        bad = int(not torch.equal(allr[lo:hi].cpu(), out.view(torch.int16).cpu()))
        gather = {"collective": "all_gather", "bytes_per_rank": 2 * n,
                  "ms": round(wdist.max_over_ranks(g_ms, coll_dev), 3),
                  "ranks_mismatched": wdist.sum_over_ranks(bad, coll_dev)}

    traffic, traffic_source = traffic_entry(args, meta, args.traffic_file)

    # The CPU baseline at every N (rank 0's host cores, its own batch), then
    # the secondary legs and the C5 strong-scaling leg -- all after the
    # headline's timed region.
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, W.batches[0]["buf"], W.shape, nbytes)
    wdist.barrier(dev)
    plan, desc, scaling = W.plan, W.desc, W.scaling
    del T, W, out
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    c2rot = c3 = c4 = rings = None
    if not args.no_extra and args.config == "c2" and not args.fused and args.kind == "ip":
        c2rot, c3, c4, rings = extra_legs(args, dev, rank, world, coll_dev)
    c5 = None
    if not args.no_c5 and args.config != "c5":
        c5 = c5_leg(args, dev, rank, world, coll_dev)
    e2e = None
    if not args.no_e2e and args.config == "c2" and not args.fused and args.kind == "ip":
        e2e = e2e_leg(args, dev, rank, world, coll_dev)

    if rank == 0:
        roof = {"bound": "hbm", "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic, "traffic_source": traffic_source,
                "frac_job": round(frac_job, 4),
                "kernel_ms_avg": round(kernel_ms, 5),
                "kernel_ms_avg_max_rank": round(kernel_ms_max, 5),
                "timing": timing}
        if frac_l3 is not None:
            roof["frac_l3_resident"] = frac_l3
        if c2rot is not None:
            roof["frac_rotating"] = c2rot["frac"]
            roof["rotating"] = c2rot
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: splitmix64 payload bytes generated on device (wc_synth_fill)"
                    + ("; well-formed IPv4 (IHL 5) / IPv6 UDP headers stamped 2:1"
                       if args.headers else "")
                    + ("; Ethernet frames with valid IPv4 header and UDP checksums"
                       if args.config in ("rx", "zrx") else ""),
            "config": {"workload": desc, **meta, "parallelism": f"packet-shard x{world}",
                       "kernel_shape": plan, "payload_GBps": round(value * GIB / 1e9, 1)},
            "roofline": roof,
            "cpu_baseline": cpu,
            "parity": parity,
            "c5": c5,
        }
        if c3 is not None:
            line["c3"] = c3
            line["c4"] = c4
        if rings is not None:
            line["rings"] = rings
        if e2e is not None:
            line["e2e"] = e2e
        if gather is not None:
            line["results_allgather"] = gather
        print(json.dumps(line), flush=True)
    if wdist._pg_active():
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())

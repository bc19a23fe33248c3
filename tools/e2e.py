#!/usr/bin/env python3
"""End-to-end (host memory in, host results out) A/B of host-path variants
(measurement tool, not product code): bench.py's `e2e` leg -- wc_cksum_host
over C2's bytes, wc_cksum_ip_udp_host (TX) and wc_rx_verdict_host (RX) over
1472-B UDP/IP packets in 2048-B netmap slots, registered and pageable, every
result checked against the oracle -- once per variant, in one process, on the
tuning build (the only one that reads the path knobs).

    python tools/e2e.py [--variants "default;WC_ZC_STREAM=0"] [--packets N] [--reps R]

One JSON line per variant: GB/s per call and memory kind, and the H2D copy
ceilings measured beside them.
"""
import argparse
import json
import os
import sys
from pathlib import Path
from types import SimpleNamespace

os.environ.setdefault("WC_TUNING", "1")  # path knobs: the tuning build reads them
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import bench  # noqa: E402
import warpcore_amd as wc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="default")
    ap.add_argument("--packets", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    wc.gpu_init(0)
    for spec in [v.strip() for v in args.variants.split(";") if v.strip()]:
        keys = []
        if spec != "default":
            for kv in spec.split():
                k, v = kv.split("=", 1)
                os.environ[k] = v
                keys.append(k)
        wc.reload_config()
        e = bench.e2e_leg(SimpleNamespace(e2e_packets=args.packets, e2e_reps=args.reps),
                          dev, 0, 1, torch.device("cpu"))
        row = {"variant": spec, "h2d_ceiling_GBps": {k: v for k, v in e["h2d_ceiling_GBps"].items()
                                                     if k != "how"}}
        for name, c in e["calls"].items():
            for kind in ("registered", "pageable"):
                row[f"{name}/{kind}"] = (c[kind]["GBps"], c[kind]["parity"]["mismatches"])
        print(json.dumps(row), flush=True)
        for k in keys:
            os.environ.pop(k)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""One line per config of a round-measurement pass (tools/round_measure.sh):
the bench line's roofline fraction (HIP events), the rocprofv3 average of the
dominant kernel and the fraction it implies, and the parity result.

    python tools/summarize_round.py <tag> cfg [cfg ...]
"""
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def main():
    tag, cfgs = sys.argv[1], sys.argv[2:]
    go = ROOT / "gpurun_out"
    for c in cfgs:
        try:
            b = json.loads((go / "round" / f"bench_{tag}_{c}.json").read_text())
            rows = list(csv.DictReader(open(go / f"prof_{tag}_{c}" / "stats" /
                                            "run_kernel_stats.csv")))
        except (OSError, ValueError) as e:
            print(f"{c:10s} missing ({e})")
            continue
        top = max(rows, key=lambda r: float(r["TotalDurationNs"]))
        avg = float(top["AverageNs"])
        r = b["roofline"]
        alg = r["achieved"] * 1e9 * r["kernel_ms_avg"] * 1e-3
        print(f"{c:10s} bench {r['frac']:.4f}  rocprof {avg / 1e3:9.2f} us = "
              f"{alg / avg:7.1f} GB/s {alg / avg / 80:5.1f} %  parity "
              f"{b['parity']['mismatches']}/{b['parity']['checked_packets']}  "
              f"{top['Name'].split('(')[0][-60:]}")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Copy one round-measurement pass (tools/round_measure.sh TAG=<tag>) from
gpurun_out/ into profiles/: bench lines, rocprofv3 kernel stats, and the HBM
traffic entries of profiles/traffic.json (tools/traffic.py; the algorithmic
bytes per launch are the workload's own, kept from the existing entry).

    python tools/collect_round.py <tag> <round> cfg [cfg ...]
"""
import json
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
KEYS = {"c2": "c2:1472", "c2pl": "c2:1472:payload:headers", "c4": "c4:zipf",
        "c4pl": "c4:zipf:payload:headers", "slots": "slots:1500",
        "slotspl": "slots:1500:payload:headers", "zslots": "zslots:zipf",
        "zslotspl": "zslots:zipf:payload:headers",
        "c2f": "c2:1472:payload:headers:fused", "c4f": "c4:zipf:payload:headers:fused",
        "slotsf": "slots:1500:payload:headers:fused",
        "zslotsf": "zslots:zipf:payload:headers:fused", "rx": "rx:1514", "zrx": "zrx:zipf", "c5": "c5:1472", "zrxa3": "zrx:zipf:arp3"}


def main():
    tag, rnd, cfgs = sys.argv[1], sys.argv[2], sys.argv[3:]
    go, prof = ROOT / "gpurun_out", ROOT / "profiles"
    traffic = json.loads((prof / "traffic.json").read_text())
    for c in cfgs:
        L = c.split("_", 1)[-1]
        key = KEYS.get(c) or ("c3:" + L + (":s2048+14" if c.startswith("s14") else "")
                              + (":payload:headers" if c.startswith(("c3pl_", "s14pl_")) else ""))
        shutil.copy(go / "round" / f"bench_{tag}_{c}.json", prof / f"bench_{rnd}_{c}.json")
        shutil.copy(go / f"prof_{tag}_{c}" / "stats" / "run_kernel_stats.csv",
                    prof / f"rocprof_{rnd}_{c}_kernel_stats.csv")
        b = json.loads((go / "round" / f"bench_{tag}_{c}.json").read_text())
        alg = traffic.get(key, {}).get("algorithmic_bytes_per_launch") or round(
            b["roofline"]["achieved"] * 1e9 * b["roofline"]["kernel_ms_avg"] * 1e-3)
        subprocess.run([sys.executable, str(ROOT / "tools" / "traffic.py"),
                        str(go / f"prof_{tag}_{c}"), key, "--algorithmic-bytes", str(alg)],
                       check=True, cwd=ROOT, stdout=subprocess.DEVNULL)
        t = json.loads((prof / "traffic.json").read_text())
        t[key]["source"] = (f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE over bench.py ({key}), "
                            f"tools/round_measure.sh TAG={tag}, round-{rnd[1:]} final kernels")
        t[key]["round"] = rnd
        (prof / "traffic.json").write_text(json.dumps(t, indent=1) + "\n")
        b = json.loads((go / "round" / f"bench_{tag}_{c}.json").read_text())
        print(f"{c:10s} frac {b['roofline']['frac']:.4f} kernel {b['roofline']['kernel_ms_avg']:.5f} ms "
              f"traffic x{t[key]['traffic_over_algorithmic']:.3f}  {t[key]['kernel']}")


if __name__ == "__main__":
    main()

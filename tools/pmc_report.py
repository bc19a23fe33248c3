#!/usr/bin/env python3
"""Summarise rocprofv3 counter_collection CSVs: per kernel name, mean of each
counter over dispatches.   python tools/pmc_report.py gpurun_out/pmc_<tag>"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1])
vals = defaultdict(lambda: defaultdict(list))
for f in root.glob("*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        short = name.split("(")[0].replace("void ", "")
        vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    if "synth" in k:
        continue
    print(f"== {k}")
    for c, v in sorted(cs.items()):
        print(f"   {c:<28} {sum(v) / len(v):16.1f}  (n={len(v)})")

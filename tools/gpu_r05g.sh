#!/usr/bin/env bash
# Round 5, call g: why the bench's every-third-ARP ring leg ran slower than
# both fixed modes (ADAPT decisions traced), then the server-interference
# and host-latency runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05g
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
for steps in 20 2000; do
  WC_RX_TRACE=1 timeout -k 10 200 python bench.py --config zrx --rx-arp 3 --no-c5 --no-extra \
      --no-cpu-baseline --steps $steps --warmup 5 > $OUT/zrxa3_$steps.json 2> $OUT/zrxa3_$steps.trace \
      || { tail -5 $OUT/zrxa3_$steps.trace; exit 1; }
  python3 - $OUT/zrxa3_$steps.json $OUT/zrxa3_$steps.trace <<'PY'
import json, re, statistics, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lines = [l for l in open(sys.argv[2]) if l.startswith("wccksum rx gen")]
early = sum("EARLY" in l for l in lines)
us = [float(re.search(r"; ([0-9.]+) us on the host", l).group(1)) for l in lines]
print(f"steps={d['steps']} kernel_ms={d['roofline']['kernel_ms_avg']} frac={d['roofline']['frac']} "
      f"launches={len(lines)} early={early} host_us_median={statistics.median(us):.1f} max={max(us):.1f}")
print("".join(lines[:3] + lines[-3:]))
PY
done
R05C_OUT=r05g bash tools/gpu_r05c.sh

#!/usr/bin/env bash
# Round 5, call ae: how often does a bench.py process put the mixed ring in
# the slow state?  Six fresh headline runs of --config zrx --rx-arp 3 (the
# config whose bench line read 152.7 us in call ac), kernel time each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05ae
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
for i in $(seq 1 6); do
  timeout -k 10 200 python bench.py --config zrx --rx-arp 3 --no-c5 --no-cpu-baseline > $OUT/b$i.json 2> $OUT/b$i.err \
      || { tail $OUT/b$i.err; exit 1; }
  python3 -c "import json; d = json.load(open('$OUT/b$i.json')); print('proc $i', d['roofline']['kernel_ms_avg'], d['roofline']['frac'])"
done

#!/usr/bin/env bash
# Round 5, call r: the zrx_arp3 leg of the default bench line read 121 us in
# call q (tune.py: 96-97 us under ADAPT).  The default line twice with every
# ADAPT decision logged (WC_RX_TRACE=1), and tune.py's zrx --rx-arp 3 beside.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05r
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
for k in 1 2; do
  WC_RX_TRACE=1 timeout -k 10 400 python bench.py --no-c5 --no-cpu-baseline > $OUT/bench$k.json 2> $OUT/bench$k.err \
      || { tail -20 $OUT/bench$k.err; exit 1; }
  python3 -c "
import json; d = json.load(open('$OUT/bench$k.json'))
print('run $k', {k: (v['kernel_ms_avg_max_rank'], v['frac']) for k, v in d['rings'].items() if isinstance(v, dict)})"
  grep -c "EARLY" $OUT/bench$k.err; grep -c ": HT" $OUT/bench$k.err
done
timeout -k 10 300 python tools/tune.py --config zrx --rx-arp 3 --rounds 3 --variants "default;WC_RX_EARLY=1;WC_RX_ADAPT=0" > $OUT/tune.log 2>&1 || exit 1
grep -E "default|WC_" $OUT/tune.log | grep -v round

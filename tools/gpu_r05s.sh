#!/usr/bin/env bash
# Round 5, call s: zrx_arp3 leg -- 121 us in call q's default line, 96.4 us
# with every ADAPT decision printed (call r).  Two plain default lines, one
# with the cheap per-512-launch summary (WC_RX_TRACE=2), and the tallying
# kernel with its decision fixed (WC_RX_FORCE=1 HT / 2 EARLY) in tune.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05s
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
for k in 1 2 3; do
  if [ $k -eq 3 ]; then export WC_RX_TRACE=2; fi
  timeout -k 10 400 python bench.py --no-c5 --no-cpu-baseline > $OUT/bench$k.json 2> $OUT/bench$k.err \
      || { tail -20 $OUT/bench$k.err; exit 1; }
  python3 -c "
import json; d = json.load(open('$OUT/bench$k.json'))
print('run $k', {k: (v['kernel_ms_avg_max_rank'], v['steps']) for k, v in d['rings'].items() if isinstance(v, dict)})"
done
unset WC_RX_TRACE
grep "rx gen" $OUT/bench3.err | tail -12
timeout -k 10 300 python tools/tune.py --config zrx --rx-arp 3 --rounds 3 \
    --variants "default;WC_RX_FORCE=1;WC_RX_FORCE=2;WC_RX_ADAPT=0;WC_RX_EARLY=1" > $OUT/tune.log 2>&1 || exit 1
grep -E "default|WC_" $OUT/tune.log | grep -v round

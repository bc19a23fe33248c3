#!/usr/bin/env bash
# Round 5, call ab: four default bench lines back to back -- the rings' spread
# with the sampled shader clock beside each leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05ab
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
for k in 1 2 3 4; do
  timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench$k.json 2> $OUT/bench$k.err || { tail -20 $OUT/bench$k.err; exit 1; }
  python3 -c "
import json; d = json.load(open('$OUT/bench$k.json'))
r = d['roofline']
print('run $k C2', r['frac'], 'rot', r['rotating']['frac'], r['rotating']['sclk_MHz'], 'C4', d['c4']['frac'], d['c4']['sclk_MHz'], 'C5', d['c5']['frac_kernel'])
print('  rings', {k: (v['kernel_ms_avg_max_rank'], v['frac'], v['sclk_MHz']) for k, v in d['rings'].items() if isinstance(v, dict)})"
done

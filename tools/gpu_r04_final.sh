#!/usr/bin/env bash
# Round-4 final measurements, in parts (each one GPU call):
#   PART=a|b|c  bash tools/gpu_r04_final.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
case ${PART:-a} in
  a) CFGS="c3_576 c3_1472 c3_9000 c4 c4pl c4f c2pl c2f" ;;
  b) CFGS="slots slotspl zslots zslotspl rx zrx" ;;
  c) CFGS="s14_64 s14pl_64 s14_128 s14pl_128 s14_256 s14pl_256" ;;
esac
CFGS="$CFGS" TAG=r04b bash tools/round_measure.sh > gpurun_out/round_r04b_${PART:-a}.log 2>&1
rc=$?
grep -h '"frac"' gpurun_out/round/bench_r04b_*.json | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']
    print(d['config']['workload'][:70], 'frac', r['frac'], 'kernel', r['kernel_ms_avg'], 'parity', d['parity'])
" || true
exit $rc

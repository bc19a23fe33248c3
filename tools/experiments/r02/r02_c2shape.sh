#!/bin/bash
# C2 and neighbours: shapes with fewer loads per lane (32- and 64-lane groups).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10 200 python tools/tune.py --rounds 4 --iters 20"
V="default;WC_SHAPE=32,4,1;WC_SHAPE=32,3,1;WC_SHAPE=32,3,2;WC_SHAPE=32,4,2;WC_SHAPE=64,2,1;WC_SHAPE=64,2,2;WC_SHAPE=32,3,4"
for L in 1472 1280 1024; do
  echo "### len $L packed"; $T --config c3 --len $L --variants "$V" 2>&1 | grep -v amdgpu.ids
done > gpurun_out/c2shape.log
for s in "" "WC_SHAPE=32,4,1" "WC_SHAPE=32,3,1" "" "WC_SHAPE=32,4,1" "WC_SHAPE=32,3,1"; do
  echo "## bench $s"; env $s timeout -k 10 120 python bench.py --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity'])"
done >> gpurun_out/c2shape.log
cat gpurun_out/c2shape.log

#!/usr/bin/env bash
# Round 5, call u: the mixed ring in bursts of 20 / 200 / 2000 launches with
# the shader clock sampled beside (tools/rx_burst.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05u
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 400 python -u tools/rx_burst.py --rounds 3 > $OUT/burst.log 2>&1 || { tail -20 $OUT/burst.log; exit 1; }
cat $OUT/burst.log

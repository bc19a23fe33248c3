#!/usr/bin/env bash
# Round 5, call t: the mixed-size ring reallocated per iteration
# (tools/rx_placement.py) -- is the intermittent slowness placement-bound?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05t
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 400 python -u tools/rx_placement.py --iters 14 > $OUT/place.log 2>&1 || { tail -20 $OUT/place.log; exit 1; }
cat $OUT/place.log
timeout -k 10 400 python -u tools/rx_placement.py --iters 8 --arp 3 > $OUT/place_arp3.log 2>&1 || { tail -20 $OUT/place_arp3.log; exit 1; }
cat $OUT/place_arp3.log

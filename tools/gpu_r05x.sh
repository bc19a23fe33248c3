#!/usr/bin/env bash
# Round 5, call x: is C4 (the dense seg path, 58 % VALU-busy in call w)
# clock-sensitive too?  rx_burst with the C4 case.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05x
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 500 python -u tools/rx_burst.py --c4 --rounds 2 --bursts 20,200,1000 > $OUT/burst.log 2>&1 || { tail -20 $OUT/burst.log; exit 1; }
cat $OUT/burst.log

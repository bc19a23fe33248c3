#!/usr/bin/env bash
# Round 5, call l: C3 shapes re-tuned from HBM (rotating buffers >= 1 GiB,
# as the bench's c3 legs run): 9000 / 576 / 256 B against neighbour shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05l
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
T="timeout -k 10 300 python tools/tune.py --rounds 4 --iters 20 --rotate-bytes $((1 << 30))"
echo "== 9000" >> $OUT/c3shapes.log
$T --config c3 --len 9000 --iters 5 --variants "default;WC_SHAPE=64,9,1;WC_SHAPE=64,9,2;WC_SHAPE=64,4,1;WC_SHAPE=32,4,1" >> $OUT/c3shapes.log 2>&1 || exit 1
echo "== 576" >> $OUT/c3shapes.log
$T --config c3 --len 576 --variants "default;WC_SHAPE=16,3,2;WC_SHAPE=16,3,4;WC_SHAPE=8,6,1;WC_SHAPE=32,2,2;WC_SHAPE=32,2,1" >> $OUT/c3shapes.log 2>&1 || exit 1
echo "== 256" >> $OUT/c3shapes.log
$T --config c3 --len 256 --variants "default;WC_SHAPE=8,2,4;WC_SHAPE=16,1,4;WC_SHAPE=16,1,8;WC_LEAN_MAX=0;WC_SHAPE=4,2,4" >> $OUT/c3shapes.log 2>&1 || exit 1
grep -E "^==|default|WC_" $OUT/c3shapes.log | grep -v "round\|rotating"

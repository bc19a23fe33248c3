#!/usr/bin/env bash
# Round 5, call y: the RX grid capped (WC_RX_GRID: several tiles per wave,
# next tile's metadata prefetched) against one tile per wave.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05y
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
V="default;WC_RX_GRID=1024;WC_RX_GRID=2048;WC_RX_GRID=4096;WC_RX_GRID=768"
timeout -k 10 300 python tools/tune.py --config zrx --rounds 4 --iters 200 --variants "$V" > $OUT/zrx.log 2>&1 || { tail $OUT/zrx.log; exit 1; }
grep -E "default|WC_" $OUT/zrx.log | grep -v round
timeout -k 10 300 python tools/tune.py --config zrx --rx-arp 3 --rounds 4 --iters 200 --variants "$V" > $OUT/zrx3.log 2>&1 || { tail $OUT/zrx3.log; exit 1; }
grep -E "default|WC_" $OUT/zrx3.log | grep -v round
timeout -k 10 300 python tools/tune.py --config rx --rounds 3 --iters 100 --variants "default;WC_RX_GRID=1024;WC_RX_GRID=2048" > $OUT/rx.log 2>&1 || { tail $OUT/rx.log; exit 1; }
grep -E "default|WC_" $OUT/rx.log | grep -v round

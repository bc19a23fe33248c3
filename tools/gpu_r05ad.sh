#!/usr/bin/env bash
# Round 5, call ad: the mixed ring's slow state is per process (bench run
# 152.7 us, the rocprof runs of the same config 96.0 us, same box).  Ten
# fresh processes, each timing ADAPT (tally stores to host memory), plain HT
# (no tally) and the plain ragged payload_cksum on the same slots.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05ad
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
for i in $(seq 1 10); do
  timeout -k 10 120 python tools/tune.py --config zrx --rounds 2 --iters 500 \
      --variants "default;WC_RX_ADAPT=0" > $OUT/p$i.log 2>&1 || { tail $OUT/p$i.log; exit 1; }
  echo "proc $i: $(grep -E '^(default|WC_)' $OUT/p$i.log | awk '{printf "%s %s us; ", $1, $2}')"
done

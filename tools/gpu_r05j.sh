#!/usr/bin/env bash
# Round 5, call j: the RX verdict kernel on the same frames in two layouts --
# one per 2048-B netmap slot (the ring) and packed back to back (C4's
# layout) -- to separate the kernel's rate from the ring layout's.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05j
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
for c in zrx rx; do
  for p in "" "--rx-packed"; do
    echo "== $c ${p:-slots}" >> $OUT/rx_layout.log
    timeout -k 10 200 python tools/tune.py --config $c $p --rounds 5 --iters 20 \
      --variants "default;WC_RX_EARLY=1" >> $OUT/rx_layout.log 2>&1 || exit 1
  done
done
grep -E "^==|default|WC_RX" $OUT/rx_layout.log | grep -v round

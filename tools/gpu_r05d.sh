#!/usr/bin/env bash
# Round 5, call d: parity of the changed paths (split launches, RX ADAPT v2,
# lean phase planner), then: C5 window / C2 / C4 with split launches
# (WC_SPLIT_PKTS), RX ADAPT v2 against fixed HT / EARLY, and call c's
# server-interference and host-latency runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05d
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -k "rx or split or lean_phase or host or fused" \
    > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/c5_window.py --windows 33554432,1048576 --allocs torch --rounds 3 \
    --variants "default;WC_SPLIT_PKTS=1048576;WC_SPLIT_PKTS=2097152;WC_SPLIT_PKTS=4194304;WC_SPLIT_PKTS=8388608" \
    > $OUT/split.log 2>&1
rc=$?; tail -11 $OUT/split.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/tune.py --config c4 --rounds 4 --iters 10 \
    --variants "default;WC_SPLIT_PKTS=2097152;WC_SPLIT_PKTS=4194304;WC_SPLIT_PKTS=8388608" \
    > $OUT/c4split.log 2>&1 || exit 1
grep -v "amdgpu.ids" $OUT/c4split.log | grep -v "^ *round"
for a in 0 3; do
  for c in zrx rx; do
    [ $c = rx ] && [ $a = 3 ] && continue
    echo "== $c arp=$a" >> $OUT/rxab.log
    timeout -k 10 200 python tools/tune.py --config $c --rx-arp $a --rounds 5 --iters 20 \
      --variants "default;WC_RX_ADAPT=0;WC_RX_EARLY=1" >> $OUT/rxab.log 2>&1 || exit 1
  done
done
grep -E "^==|default|WC_RX" $OUT/rxab.log | grep -v round
bash tools/gpu_r05c.sh

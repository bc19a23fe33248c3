#!/usr/bin/env bash
# Round 5, call b: the full GPU suite (new: fused host call, server stats and
# heartbeat, TX queue hook, RX modes incl. SKIP, merged lean phase path),
# the C5 clock probe, then the lean phase path's A/B (WC_LEAN_PHASE=0 is the
# round-4 planner) on rotating buffers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05b
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/c5_clock.py --rounds 3 > $OUT/c5clock.log 2>&1
rc=$?; tail -9 $OUT/c5clock.log; [ $rc -eq 0 ] || exit $rc
T="timeout -k 10 200 python tools/tune.py --rounds 4 --iters 20 --rotate-bytes $((1 << 30))"
for L in 64 128 256 576; do
  for k in ip payload; do
    h=""; [ $k = payload ] && h="--headers"
    echo "== s14-$L $k" >> $OUT/leanph.log
    $T --config c3 --len $L --stride 2048 --offset 14 --kind $k $h \
      --variants "default;WC_LEAN_PHASE=0" >> $OUT/leanph.log 2>&1 || exit 1
  done
done
grep -v "amdgpu.ids" $OUT/leanph.log | grep -E "^==|default|PHASE"
# RX verdict: the ADAPT default against the fixed HT (WC_RX_ADAPT=0) and
# EARLY modes, all-UDP and every-third-frame-ARP mixed rings, the MTU ring
for a in 0 3; do
  for c in zrx rx; do
    [ $c = rx ] && [ $a = 3 ] && continue
    echo "== $c arp=$a" >> $OUT/rxab.log
    timeout -k 10 200 python tools/tune.py --config $c --rx-arp $a --rounds 5 --iters 20 \
      --variants "default;WC_RX_ADAPT=0;WC_RX_EARLY=1" >> $OUT/rxab.log 2>&1 || exit 1
  done
done
grep -E "^==|default|WC_RX" $OUT/rxab.log | grep -v round

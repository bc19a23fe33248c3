#!/usr/bin/env bash
# Round-4 pass d: RX EARLY at 5 waves/SIMD (in-tree) vs 4 (tools/libwccksum_prev.so),
# then the round measurement of C3 64/128/256 B on rotating buffers and C2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04d
mkdir -p $O
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "early or host_ or rx_verdict_host or c_rx or c_host" > $O/t_rx.log 2>&1 || { tail -30 $O/t_rx.log; exit 1; }
tail -1 $O/t_rx.log
for W in 64 128; do
  WC_SERVE_WAVES=$W timeout -k 10 200 build/host_latency 16 0.2 > $O/host_latency_w$W.log 2>&1 || { tail $O/host_latency_w$W.log; exit 1; }
  echo "== waves $W"; cut -c1-150 $O/host_latency_w$W.log | head -4; sed -n 7,10p $O/host_latency_w$W.log | cut -c1-150
done
T="python tools/tune.py --rounds 4 --iters 20 --warm-ms 50"
for a in "--config zrx" "--config rx" "--config zrx --rx-arp 3"; do
  echo "== $a" | tee -a $O/ab.log
  for rep in 1 2; do
    echo -n "prev " | tee -a $O/ab.log; WC_LIB=tools/libwccksum_prev.so timeout -k 10 120 $T $a --variants "WC_RX_SKIP=0;WC_RX_EARLY=1" 2>&1 | grep -v amdgpu | tee -a $O/ab.log || exit 1
    echo -n "new  " | tee -a $O/ab.log; timeout -k 10 120 $T $a --variants "WC_RX_SKIP=0;WC_RX_EARLY=1" 2>&1 | grep -v amdgpu | tee -a $O/ab.log || exit 1
  done
done
CFGS="c3_64 c3_128 c3_256 c2" TAG=r04a bash tools/round_measure.sh > $O/round.log 2>&1 || { tail -20 $O/round.log; exit 1; }
grep -v "^==" $O/round.log | tail -8

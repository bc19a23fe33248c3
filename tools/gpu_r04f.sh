#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04f
mkdir -p $O
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "resident or rx_verdict_host or c_rx or c_host" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for W in 64 128; do
  WC_SERVE_WAVES=$W timeout -k 10 200 build/host_latency 16 0.3 > $O/host_latency_w$W.log 2>&1 || { tail $O/host_latency_w$W.log; exit 1; }
  echo "== waves $W"; cut -c1-130 $O/host_latency_w$W.log | head -4; sed -n 7,10p $O/host_latency_w$W.log | cut -c1-130
done

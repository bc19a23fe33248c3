#!/usr/bin/env bash
# Round-4 second pass: RX kernel modes (transposed header loads, skip),
# their parity in every mode, and the C4 result-store PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04b
mkdir -p $O
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_rx.py -x -q --timeout 300 --timeout-method thread > $O/t_rx.log 2>&1 || { tail -40 $O/t_rx.log; exit 1; }
tail -2 $O/t_rx.log
timeout -k 10 120 build/rx_ring_loop 4 1024 > $O/rx_ring.log 2>&1 || { cat $O/rx_ring.log; exit 1; }
V="WC_RX_HDRT=0 WC_RX_SKIP=0;WC_RX_SKIP=0;default;WC_RX_EARLY=1 WC_RX_HDRT=0;WC_RX_EARLY=1"
for a in "--config zrx" "--config rx" "--config zrx --rx-arp 3"; do
  echo "== tune $a" >> $O/tune_rx.log
  timeout -k 10 200 python tools/tune.py $a --rounds 5 --iters 20 --variants "$V" >> $O/tune_rx.log 2>&1 || exit 1
done
grep -v amdgpu $O/tune_rx.log
TAG=c4 bash tools/pmc_store.sh > $O/pmc_store.log 2>&1 || { tail -20 $O/pmc_store.log; exit 1; }
cat $O/pmc_store.log | grep -v "rc=0"

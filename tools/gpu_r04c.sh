#!/usr/bin/env bash
# Round-4 third pass: the whole -m gpu suite on the block-delegated result
# stores, then A/B of the previous build (tools/libwccksum_prev.so) against
# the in-tree one, alternating, per config.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04c
mkdir -p $O
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_all.log 2>&1 || { tail -40 $O/t_all.log; exit 1; }
tail -2 $O/t_all.log
T="python tools/tune.py --rounds 4 --iters 20 --warm-ms 50"
for a in "--config c2" "--config c4" "--config c4 --kind payload --headers" "--config c4 --fused --headers --kind payload" "--config c3 --len 64" "--config c3 --len 256" "--config c3 --len 1472 --stride 2048 --offset 14" "--config zslots" "--config zrx" "--config rx"; do
  echo "== $a" | tee -a $O/ab.log
  for rep in 1 2; do
    echo -n "prev " | tee -a $O/ab.log; WC_LIB=tools/libwccksum_prev.so timeout -k 10 120 $T $a 2>&1 | grep -v amdgpu | tee -a $O/ab.log || exit 1
    echo -n "new  " | tee -a $O/ab.log; timeout -k 10 120 $T $a 2>&1 | grep -v amdgpu | tee -a $O/ab.log || exit 1
  done
done

#!/usr/bin/env bash
# Seg-only packed strided payload_cksum (per-lane exact fallback, no flat path) = new vs prev build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/sp_pytest.log 2>&1 || { tail -40 gpurun_out/sp_pytest.log; exit 1; }
tail -1 gpurun_out/sp_pytest.log
T="timeout -k 10 120 python tools/tune.py --rounds 3 --iters 20 --warm-ms 20 --kind payload"
for L in 64 100 256 576 900; do
  for h in --headers ""; do
    for rep in 1 2; do
      echo -n "prev $L $h: "; WC_LIB=tools/libwccksum_prev.so $T --config c3 --len $L $h 2>&1 | grep -v amdgpu.ids || exit 1
      echo -n "new  $L $h: "; $T --config c3 --len $L $h 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done

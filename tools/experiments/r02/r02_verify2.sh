#!/bin/bash
# Strided parity, then bench lines for C2 ip / payload and strided slots.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "strided or c2 or c3 or slot" --timeout 240 --timeout-method thread \
    > gpurun_out/verify2_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/verify2_pytest.log
[ $rc -eq 0 ] || exit $rc
T="timeout -k 10 200 python tools/tune.py --rounds 4 --iters 20"
for a in "--config c2" "--config c2 --kind payload --headers" "--config c3 --len 1500 --stride 2048 --offset 14" "--config c3 --len 1500 --stride 2048 --offset 14 --kind payload --headers" "--config c3 --len 1024 --kind payload --headers" "--config c3 --len 1000 --stride 2048 --offset 14 --kind payload --headers"; do
  echo "## $a"; $T $a --variants "default;WC_SHAPE=16,6,4" 2>&1 | grep -v amdgpu.ids
done

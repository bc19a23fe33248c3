#!/bin/bash
# Strided parity after the small-size planner tweaks, then C3 sizes and the
# large-packet shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "strided or c3" --timeout 240 --timeout-method thread \
    > gpurun_out/verify3_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/verify3_pytest.log
[ $rc -eq 0 ] || exit $rc
T="timeout -k 10 200 python tools/tune.py --rounds 4 --iters 20"
for L in 64 256 320 576 704 1472; do echo "## len $L"; $T --config c3 --len $L 2>&1 | grep -v amdgpu.ids; done
for L in 2048 3000 4096 9000; do
  echo "## len $L"; $T --config c3 --len $L --variants "default;WC_SHAPE=32,18,1;WC_SHAPE=64,9,1;WC_SHAPE=64,9,2;WC_SHAPE=64,4,1;WC_SHAPE=32,4,1" 2>&1 | grep -v amdgpu.ids
done

#!/usr/bin/env bash
# (4,1,4): group g takes packets g U + u (each lane stores its own packet's result) vs u GPW + g + exchange.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/os_pytest.log 2>&1 || { tail -40 gpurun_out/os_pytest.log; exit 1; }
tail -1 gpurun_out/os_pytest.log
T="timeout -k 10 120 python tools/tune.py --rounds 6 --iters 20 --warm-ms 20"
echo "### c3 64 ip"; $T --config c3 --len 64 --variants "WC_VARIANT=2097152;default" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### c3 48 ip"; $T --config c3 --len 48 --variants "WC_VARIANT=2097152;default" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### 64 in 2048 slots +14 ip"; $T --config c3 --len 64 --stride 2048 --offset 14 --variants "WC_VARIANT=2097152;default" 2>&1 | grep -v amdgpu.ids || exit 1

#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
WC_VARIANT=131072 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "strided or ragged or golden or zslots or c4" \
    > gpurun_out/al_pytest.log 2>&1 || { tail -40 gpurun_out/al_pytest.log; exit 1; }
tail -1 gpurun_out/al_pytest.log
T="timeout -k 10 120 python tools/tune.py --rounds 4 --iters 20 --warm-ms 20"
for L in 300 1000 1300; do echo "### c3 $L packed (seg, STR ip)"; $T --config c3 --len $L --variants "default;WC_VARIANT=131072" 2>&1 | grep -v amdgpu.ids || exit 1; done
echo "### c4 ip"; $T --config c4 --variants "default;WC_VARIANT=131072" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### c4 payload+h"; $T --config c4 --kind payload --headers --variants "default;WC_VARIANT=131072" 2>&1 | grep -v amdgpu.ids || exit 1

#!/usr/bin/env bash
# A/B of strided-kernel variants (WC_VARIANT) on the GPU box; parity first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
V=${V:-1}
WC_VARIANT=$V timeout -k 10 300 python -m pytest tests -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -2 gpurun_out/ab_pytest.log
T="timeout -k 10 200 python tools/tune.py --rounds 6 --iters 20"
$T --config c2 --kind payload --variants "default;WC_VARIANT=$V" > gpurun_out/ab_c2_payload.log 2>&1 &&
$T --config c3 --len 1500 --stride 2048 --offset 14 --kind ip --variants "default;WC_VARIANT=$V" > gpurun_out/ab_slot_ip.log 2>&1 &&
$T --config c3 --len 1500 --stride 2048 --offset 14 --kind payload --variants "default;WC_VARIANT=$V" > gpurun_out/ab_slot_payload.log 2>&1 &&
$T --config c2 --kind ip --variants "default;WC_VARIANT=$V" > gpurun_out/ab_c2_ip.log 2>&1
rc=$?
cat gpurun_out/ab_*.log | grep -v "^\s*round"
exit $rc

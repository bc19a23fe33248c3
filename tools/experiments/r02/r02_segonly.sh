#!/usr/bin/env bash
# Seg-only packed strided ip_cksum kernel (5 / 7 waves per SIMD): parity of the strided tests, then A/B vs prev build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "strided or planner or golden or kat" \
    > gpurun_out/so_pytest.log 2>&1 || { tail -40 gpurun_out/so_pytest.log; exit 1; }
tail -1 gpurun_out/so_pytest.log
CASES="c3-100:ip c3-144:ip c3-200:ip c3-300:ip c3-700:ip c3-1000:ip" ROUNDS=3 bash tools/ab_lib.sh

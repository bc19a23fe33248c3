#!/usr/bin/env bash
# payload group kernel: DPP header broadcast (default) vs ds_bpermute exchange (WC_VARIANT bit 19).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/hd_pytest.log 2>&1 || { tail -40 gpurun_out/hd_pytest.log; exit 1; }
tail -1 gpurun_out/hd_pytest.log
T="timeout -k 10 120 python tools/tune.py --rounds 4 --iters 20 --warm-ms 20 --kind payload --headers"
echo "### c2 payload"; $T --config c2 --variants "WC_VARIANT=524288;default" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### slots 1500 +14 payload strided"; $T --config c3 --len 1500 --stride 2048 --offset 14 --variants "WC_VARIANT=524288;default" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### 1024 +14 stride 2048 payload strided"; $T --config c3 --len 1024 --stride 2048 --offset 14 --variants "WC_VARIANT=524288;default" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### 9000 payload"; $T --config c3 --len 9000 --packets 131072 --variants "WC_VARIANT=524288;default" 2>&1 | grep -v amdgpu.ids || exit 1

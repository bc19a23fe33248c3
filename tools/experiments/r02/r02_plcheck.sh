#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/plc_pytest.log 2>&1 || { tail -40 gpurun_out/plc_pytest.log; exit 1; }
tail -1 gpurun_out/plc_pytest.log
T="timeout -k 10 120 python tools/tune.py --rounds 4 --iters 20 --warm-ms 20 --kind payload --headers"
for L in 64 256 576 1472; do echo "### payload $L"; $T --config c3 --len $L --variants "default;WC_STRIDED_SEG=0" 2>&1 | grep -v amdgpu.ids || exit 1; done

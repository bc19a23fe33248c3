#!/bin/bash
# Flat fallback with word sums (WC_VARIANT=32): ragged parity, then A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "vsum or zslots or ragged or dense" --timeout 240 --timeout-method thread \
    > gpurun_out/vsum_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/vsum_pytest.log
[ $rc -eq 0 ] || exit $rc
T="timeout -k 10 200 python tools/tune.py --rounds 5 --iters 20"
echo "## zslots ip"; $T --config zslots --variants "default;WC_VARIANT=32;default;WC_VARIANT=32" 2>&1 | grep -v amdgpu.ids
echo "## c4 ip (no flat tiles)"; $T --config c4 --variants "default;WC_VARIANT=32" 2>&1 | grep -v amdgpu.ids
echo "## c4 ip, flat forced via seg fallback (WC_GRP_SPARSE=65, random placement: ragged sweep)"; $T --config zslots --packets 524288 --variants "default;WC_VARIANT=32" 2>&1 | grep -v amdgpu.ids

#!/bin/bash
# Full GPU parity suite, then a two-build A/B (tools/libwccksum_prev.so vs
# the in-tree build) over CASES.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/check_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/check_pytest.log
[ $rc -eq 0 ] || exit $rc
CASES="${CASES:-c3-64:ip c3-128:ip c3-256:ip c3-576:ip c2:ip c3-9000:ip c4:ip slot:ip}" ROUNDS=${ROUNDS:-3} \
    bash tools/ab_lib.sh > gpurun_out/check_ab.log 2>&1
grep -v amdgpu gpurun_out/check_ab.log

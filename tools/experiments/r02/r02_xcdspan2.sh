#!/usr/bin/env bash
# seg kernel default XCD span 2^13 (default) vs the previous 2^12 (WC_VARIANT=3072), then C4/zslots parity.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/xs_pytest.log 2>&1 || { tail -40 gpurun_out/xs_pytest.log; exit 1; }
tail -1 gpurun_out/xs_pytest.log
CASES="c4:ip c4:payload+h rslot:payload+h zslots:ip zslots:payload+h rc2:ip" VARS="WC_VARIANT=3072;default" ROUNDS=4 bash tools/ab.sh

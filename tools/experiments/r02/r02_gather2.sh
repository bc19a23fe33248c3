#!/usr/bin/env bash
# Gathered path: parity (ragged tests in every mode, incl. forced gather), A/B on random order.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gather_pytest.log 2>&1 || { tail -40 gpurun_out/gather_pytest.log; exit 1; }
tail -1 gpurun_out/gather_pytest.log
CASES="c4r:ip c4r:payload+h zslots:ip zslots:payload" VARS="WC_GATHER=0;default;WC_GATHER=2" ROUNDS=4 bash tools/ab.sh

#!/usr/bin/env bash
# Gathered-stream path of k_cksum_seg: full GPU parity, then A/B against the
# flat fallback (WC_GATHER=0) on the mixed-size ring, C4 and random placement.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gather_pytest.log 2>&1 || { tail -40 gpurun_out/gather_pytest.log; exit 1; }
tail -1 gpurun_out/gather_pytest.log
CASES=${CASES:-"zslots:ip zslots:payload+h c4:ip rc2:ip"} VARS=${VARS:-"WC_GATHER=0;default"} \
    ROUNDS=${ROUNDS:-5} bash tools/ab.sh

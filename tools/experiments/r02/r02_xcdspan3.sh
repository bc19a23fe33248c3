#!/usr/bin/env bash
# strided kernel XCD span: 2^12 (default) vs 2^11 / 2^13 / 2^14.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
CASES="c2:ip c2:payload+h c3-64:ip c3-256:ip c3-9000:ip slot:ip" VARS="default;WC_VARIANT=2816;WC_VARIANT=3328;WC_VARIANT=3584" ROUNDS=4 bash tools/ab.sh

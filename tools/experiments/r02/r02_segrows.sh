#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
T="timeout -k 10 120 python tools/tune.py --rounds 4 --iters 20 --warm-ms 20"
for L in 300 1000 1300; do echo "### c3 $L packed (seg, STR ip)"; $T --config c3 --len $L --variants "default;WC_SEG_ROWS=2;WC_SEG_ROWS=8" 2>&1 | grep -v amdgpu.ids || exit 1; done
echo "### c4 ip"; $T --config c4 --variants "default;WC_SEG_ROWS=2;WC_SEG_ROWS=8" 2>&1 | grep -v amdgpu.ids || exit 1

#!/bin/bash
# C4 seg-kernel knobs (rows per group, grid) on the round-2 build.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "planner_shapes" --timeout 120 --timeout-method thread 2>&1 | tail -2
T="timeout -k 10 200 python tools/tune.py --rounds 4 --iters 10"
$T --config c4 --variants "default;WC_SEG_ROWS=2;WC_SEG_ROWS=8;WC_GRP_ROWS=2;WC_NT=0" 2>&1 | grep -v amdgpu.ids
$T --config c4 --kind payload --headers --variants "default;WC_SEG_ROWS=2;WC_SEG_ROWS=8" 2>&1 | grep -v amdgpu.ids

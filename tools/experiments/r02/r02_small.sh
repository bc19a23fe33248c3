#!/bin/bash
# Round 2: small packed packets (C3 64 B, 100 B, 128 B) -- strided shapes,
# grid caps and the seg kernel, interleaved A/B with the read-stream ceiling.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10 150 python tools/tune.py --rounds 5 --iters 40"
$T --config c3 --len 64 --variants "default;WC_SHAPE=4,1,1;WC_SHAPE=4,1,2;WC_SHAPE=4,1,8;WC_SHAPE=4,1,2 WC_BLOCKS_PER_CU=32;WC_SHAPE=4,1,4 WC_BLOCKS_PER_CU=16" > gpurun_out/small_64.log 2>&1
$T --config c3 --len 100 --variants "default;WC_STRIDED_SEG=0;WC_STRIDED_SEG=0 WC_SHAPE=8,1,2;WC_STRIDED_SEG=0 WC_SHAPE=8,1,4;WC_STRIDED_SEG=0 WC_SHAPE=4,2,2;WC_SEG_ROWS=4" > gpurun_out/small_100.log 2>&1
$T --config c3 --len 128 --variants "default;WC_SHAPE=8,1,2;WC_SHAPE=8,1,8;WC_SHAPE=4,2,2;WC_SHAPE=4,2,4" > gpurun_out/small_128.log 2>&1
grep -v amdgpu.ids gpurun_out/small_*.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k capped_grid --timeout 240 --timeout-method thread > gpurun_out/capped.log 2>&1; tail -3 gpurun_out/capped.log

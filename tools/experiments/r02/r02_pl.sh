#!/bin/bash
set -e
export WC_NO_BUILD=1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "ragged or payload or fused or zslots or c4 or host" > gpurun_out/pl_parity.log 2>&1
T="timeout -k 10 150 python tools/tune.py --rounds 5 --iters 20"
$T --config zslots --kind payload --headers --variants "default;WC_SEG=0" > gpurun_out/pl_zslots.log 2>&1
$T --config zslots --variants "default;WC_SEG=0" > gpurun_out/ip_zslots.log 2>&1
$T --config c4 --kind payload --variants "default;WC_SEG=0" > gpurun_out/pl_c4r.log 2>&1
$T --config c3 --len 64 --variants "default;WC_SHAPE=4,1,2;WC_SHAPE=4,1,8;WC_SHAPE=8,1,2;WC_VARIANT=8;WC_BLOCKS_PER_CU=8;WC_BLOCKS_PER_CU=16" > gpurun_out/t64.log 2>&1
$T --config c3 --len 256 --offset 14 --variants "default;WC_STRIDED_SEG=0;WC_SEG_ROWS=2;WC_SEG_ROWS=8" > gpurun_out/t256o14.log 2>&1
$T --config c3 --len 100 --variants "default;WC_STRIDED_SEG=0;WC_SEG_ROWS=2;WC_SEG_ROWS=8" > gpurun_out/t100.log 2>&1

#!/bin/bash
# Grouped-path (size classes) check: ragged parity, then zslots / slots / c4 timings.
set -e
export WC_NO_BUILD=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "ragged or payload or fused or zslots or c4" > gpurun_out/grp_parity.log 2>&1
T="timeout -k 10 150 python tools/tune.py --rounds 5 --iters 20"
V="default;WC_GRP_SPARSE=0;WC_GRP_SPARSE=24;WC_GRP_SPARSE=32;WC_GRP_SPARSE=48;WC_SEG=0"
$T --config zslots --variants "$V" > gpurun_out/zslots_ip.log 2>&1
$T --config zslots --kind payload --headers --variants "$V" > gpurun_out/zslots_pl.log 2>&1
$T --config c4 --variants "default;WC_SEG=0" > gpurun_out/c4.log 2>&1
$T --config c3 --len 1472 --offset 14 --stride 2048 --ragged --variants "default;WC_GRP_SPARSE=65" > gpurun_out/slots.log 2>&1
$T --config c3 --len 1472 --offset 14 --stride 2048 --ragged --kind payload --headers --variants "default;WC_GRP_SPARSE=65" > gpurun_out/slots_pl.log 2>&1

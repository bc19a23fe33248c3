#!/bin/bash
set -e
export WC_NO_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "ragged or payload or fused or zslots or c4 or strided or c3 or c2" > gpurun_out/tail_parity.log 2>&1
T="timeout -k 10 150 python tools/tune.py --rounds 5 --iters 20"
$T --config c4 --variants "default;WC_SEG_ROWS=2;WC_SEG=0" > gpurun_out/tail_c4.log 2>&1
$T --config c4 --kind payload --headers --variants "default;WC_SEG_ROWS=2" > gpurun_out/tail_c4pl.log 2>&1
$T --config zslots --variants "default;WC_SEG=0" > gpurun_out/tail_zslots.log 2>&1
$T --config zslots --kind payload --headers --variants "default;WC_SEG=0" > gpurun_out/tail_zslotspl.log 2>&1
$T --config c3 --len 1472 --offset 14 --stride 2048 --ragged --variants "default" > gpurun_out/tail_slots.log 2>&1
for a in "--len 256 --offset 14" "--len 100" "--len 300" "--len 120 --offset 14" "--len 800 --offset 14"; do
  echo "## $a"; $T --config c3 $a --variants "default;WC_STRIDED_SEG=0"
done > gpurun_out/tail_c3.log 2>&1
$T --config c2 --variants "default" > gpurun_out/tail_c2.log 2>&1

#!/bin/bash
# Packed strided batches at unaligned lengths / offsets: group kernel vs the
# seg kernel (STR) with 2 / 4 rows per group -- re-tunes the planner's
# WC_STRIDED_SEG size window (wc_cksum_api.cpp plan_strided).
set -e
export WC_NO_BUILD=1
mkdir -p gpurun_out
V="default;WC_STRIDED_SEG=0;WC_STRIDED_SEG=2 WC_SEG_ROWS=2;WC_STRIDED_SEG=2"
for off in 0 14; do
  for L in 60 100 130 200 256 300 400 500 576 700 1000 1472; do
    echo "### len $L offset $off"
    timeout -k 10 120 python tools/tune.py --config c3 --len $L --offset $off --rounds 3 --iters 20 --variants "$V" | grep -v "^ *round\|amdgpu.ids"
  done
done

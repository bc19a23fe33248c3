#!/bin/bash
# Packed strided batches (stride = len) at offsets 0 and 14: the group kernel
# against the seg kernel with 2 and 4 rows per group, 30 lengths -- the data
# behind plan_strided's kernel choice (wc_cksum_api.cpp).
set -e
export WC_NO_BUILD=1
V="WC_STRIDED_SEG=0;WC_STRIDED_SEG=2 WC_SEG_ROWS=2;WC_STRIDED_SEG=2 WC_SEG_ROWS=4"
for off in 0 14; do
  for L in 40 64 80 100 120 150 180 200 220 240 256 270 300 330 360 400 450 500 550 576 600 650 700 760 800 900 1000 1100 1200 1300; do
    echo "### len $L offset $off"
    timeout -k 10 120 python tools/tune.py --config c3 --len $L --offset $off --rounds 3 --iters 20 --warm-ms 20 --variants "$V" | grep -v "^ *round\|amdgpu.ids"
  done
done

#!/usr/bin/env bash
# Packed strided batches 64..320 B: group kernel vs seg kernel (2 / 4 rows), aligned sizes
# included (WC_VARIANT=2 lets an aligned batch take the seg path); C3 64 B store / grid probes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
T="timeout -k 10 120 python tools/tune.py --rounds 4 --iters 20 --warm-ms 20"
out=gpurun_out/s3.log; : > $out
echo "### c3 64 probes" | tee -a $out
$T --config c3 --len 64 --variants "default;WC_VARIANT=64;WC_BLOCKS_PER_CU=16;WC_BLOCKS_PER_CU=32;WC_SHAPE=4,1,2 WC_BLOCKS_PER_CU=32;WC_SHAPE=4,1,2 WC_VARIANT=64" 2>&1 | grep -v "amdgpu.ids" | tee -a $out || exit 1
V="default;WC_STRIDED_SEG=0;WC_VARIANT=2 WC_STRIDED_SEG=2 WC_SEG_ROWS=2;WC_VARIANT=2 WC_STRIDED_SEG=2 WC_SEG_ROWS=4"
for off in 0 14; do
  for L in 64 80 96 100 112 120 128 144 150 160 176 192 200 208 224 240 256 288 320; do
    echo "### len $L offset $off" | tee -a $out
    $T --config c3 --len $L --offset $off --variants "$V" 2>&1 | grep -v "amdgpu.ids" | tee -a $out || exit 1
  done
done

#!/bin/bash
# 49..96-chunk packets: (16,4,U) / (16,5,U) shapes vs the planner's (16,6,4).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10 200 python tools/tune.py --rounds 4 --iters 20"
for L in 800 1024 1200 1280; do
  $T --config c3 --len $L --variants "default;WC_SHAPE=16,4,4;WC_SHAPE=16,4,2;WC_SHAPE=16,5,4;WC_SHAPE=16,5,2;WC_SHAPE=32,3,4;WC_SHAPE=32,4,1" > gpurun_out/mid_$L.log 2>&1
  $T --config c3 --len $L --offset 14 --stride 2048 --variants "default;WC_SHAPE=16,4,4;WC_SHAPE=16,5,4;WC_SHAPE=16,5,2" > gpurun_out/mid_${L}_slot.log 2>&1
done
for f in gpurun_out/mid_*.log; do echo "## $f"; grep -v amdgpu.ids $f; done

#!/bin/bash
# Netmap slot rings (ragged) through the ragged group kernel (one packet per
# 16/32/64-lane group, WC_FLAT_MIN forces it) vs the seg kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10 200 python tools/tune.py --rounds 4 --iters 20"
G="WC_FLAT_MIN=1000000000000"
V="default;$G WC_RAGGED_SHAPE=32,4,1;$G WC_RAGGED_SHAPE=32,3,2;$G WC_RAGGED_SHAPE=64,2,1;$G WC_RAGGED_SHAPE=16,6,4"
for L in 1500 1000; do
  echo "## ragged slots len $L ip"; $T --config c3 --len $L --stride 2048 --offset 14 --ragged --variants "$V" 2>&1 | grep -v amdgpu.ids
  echo "## ragged slots len $L payload+h"; $T --config c3 --len $L --stride 2048 --offset 14 --ragged --kind payload --headers --variants "$V" 2>&1 | grep -v amdgpu.ids
done
echo "## zslots"; $T --config zslots --variants "$V" 2>&1 | grep -v amdgpu.ids

#!/bin/bash
# Round 2: strided shapes for 49..97-chunk packets (784..1536 B), packed
# aligned (stride = len) and in 2048-B slots at +14; tune.py, interleaved.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10 200 python tools/tune.py --rounds 3 --iters 20"
V="default;WC_SHAPE=16,4,4;WC_SHAPE=16,5,4;WC_SHAPE=32,3,4;WC_SHAPE=32,4,1;WC_SHAPE=16,6,4"
for L in 784 848 912 976 1040 1104 1168 1232 1296 1360 1424 1472 1536; do
  echo "### len $L packed"
  $T --config c3 --len $L --variants "$V" 2>&1 | grep -v amdgpu.ids
  echo "### len $L slot+14"
  $T --config c3 --len $L --offset 14 --stride 2048 --variants "$V" 2>&1 | grep -v amdgpu.ids
done > gpurun_out/sweep_mid.log
cat gpurun_out/sweep_mid.log

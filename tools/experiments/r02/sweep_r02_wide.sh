#!/bin/bash
# Round 2: strided shapes with 32-lane groups vs the planner for 49..97-chunk
# packets, packed aligned (stride = len) and in 2048-B slots at +14.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10 200 python tools/tune.py --rounds 3 --iters 20"
V="default;WC_SHAPE=16,4,4;WC_SHAPE=16,5,4;WC_SHAPE=32,2,2;WC_SHAPE=32,2,4;WC_SHAPE=32,3,1;WC_SHAPE=32,3,2;WC_SHAPE=32,4,1;WC_SHAPE=32,4,2"
for L in ${LENS:-784 816 848 880 912 944 976 1008 1024 1056 1088 1120 1152 1184 1216 1248 1280 1312 1344 1376 1408 1440 1472 1504 1536}; do
  echo "### len $L packed"
  $T --config c3 --len $L --variants "$V" 2>&1 | grep -v amdgpu.ids
  echo "### len $L slot+14"
  $T --config c3 --len $L --offset 14 --stride 2048 --variants "$V" 2>&1 | grep -v amdgpu.ids
done > gpurun_out/sweep_wide.log
tail -2 gpurun_out/sweep_wide.log

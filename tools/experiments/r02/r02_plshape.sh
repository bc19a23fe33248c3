#!/bin/bash
# payload_cksum strided shapes for 49..97-chunk packets (C2 payload, slots).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10 200 python tools/tune.py --rounds 3 --iters 20 --kind payload --headers"
V="default;WC_SHAPE=16,6,4;WC_SHAPE=16,5,4;WC_SHAPE=16,4,4;WC_SHAPE=32,3,1;WC_SHAPE=32,3,2;WC_SHAPE=32,4,2;WC_SHAPE=16,6,2"
for L in 800 1024 1200 1472; do
  echo "### len $L packed payload"; $T --config c3 --len $L --variants "$V" 2>&1 | grep -v amdgpu.ids
  echo "### len $L slot+14 payload"; $T --config c3 --len $L --offset 14 --stride 2048 --variants "$V" 2>&1 | grep -v amdgpu.ids
done > gpurun_out/plshape.log
cat gpurun_out/plshape.log

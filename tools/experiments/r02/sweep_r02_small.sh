#!/bin/bash
# Round 2: strided shapes for 9..48-chunk packets (144..768 B), aligned packed
# (FULL) and 2048-B slots at +14 (masked), ip_cksum.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10 200 python tools/tune.py --rounds 3 --iters 20"
V="default;WC_SHAPE=8,3,2;WC_SHAPE=16,1,4;WC_SHAPE=16,2,2;WC_SHAPE=16,2,4;WC_SHAPE=16,3,1;WC_SHAPE=16,3,2;WC_SHAPE=32,1,2;WC_SHAPE=32,1,4;WC_SHAPE=32,2,1;WC_SHAPE=8,6,1"
for L in ${LENS:-144 192 256 320 384 448 512 576 640 704 768}; do
  echo "### len $L packed"
  $T --config c3 --len $L --variants "$V" 2>&1 | grep -v amdgpu.ids
  echo "### len $L slot+14"
  $T --config c3 --len $L --offset 14 --stride 2048 --variants "$V" 2>&1 | grep -v amdgpu.ids
done > gpurun_out/sweep_small.log
tail -2 gpurun_out/sweep_small.log

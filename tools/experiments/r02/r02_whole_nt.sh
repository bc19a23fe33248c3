#!/bin/bash
# whole-chunk flat tiles with temporal stream loads (edge re-loads then hit L2)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10 150 python tools/tune.py --rounds 5 --iters 20"
V="WC_SEG=0;WC_SEG=0 WC_NT=0;WC_SEG=0 WC_NT=0 WC_WALK=4096;WC_SEG=0 WC_WALK=4096"
$T --config zslots --variants "$V" > gpurun_out/whole_nt_zslots.log 2>&1
$T --config c4 --variants "$V" > gpurun_out/whole_nt_c4.log 2>&1
timeout -k 10 100 python tools/tune.py --config c3 --len 64 --ceiling > gpurun_out/c3_64_ceiling.log 2>&1
timeout -k 10 100 python tools/tune.py --config c3 --len 100 --ceiling > gpurun_out/c3_100_ceiling.log 2>&1
cat gpurun_out/whole_nt_*.log gpurun_out/c3_*_ceiling.log | grep -v amdgpu.ids

#!/bin/bash
# Round 2: lane-pattern probe with misaligned blocks; flat PK=2 on zslots.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/pattern_probe.py --rounds 3 > gpurun_out/pattern2.log 2>&1
T="timeout -k 10 150 python tools/tune.py --rounds 5 --iters 20"
V="WC_SEG=0;WC_SEG=0 WC_FLAT_PK=2;WC_SEG=0 WC_FLAT_UN=4;WC_SEG=0 WC_FLAT_UN=1;default"
$T --config zslots --variants "$V" > gpurun_out/pk2_zslots_ip.log 2>&1
cat gpurun_out/pattern2.log gpurun_out/pk2_zslots_ip.log | grep -v amdgpu.ids

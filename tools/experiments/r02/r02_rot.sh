#!/bin/bash
# C2 with the chunk -> lane map rotated by 1..8 chunks (WC_VARIANT = 16 | rot << 16).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10 200 python tools/tune.py --rounds 5 --iters 20"
V="default;WC_VARIANT=$((16|1<<16));WC_VARIANT=$((16|2<<16));WC_VARIANT=$((16|4<<16));WC_VARIANT=$((16|8<<16));WC_VARIANT=$((16|16<<16))"
$T --config c2 --variants "$V" > gpurun_out/rot_c2.log 2>&1
$T --config c3 --len 1024 --variants "$V" > gpurun_out/rot_1024.log 2>&1
$T --config c3 --len 512 --variants "$V" > gpurun_out/rot_512.log 2>&1
grep -v amdgpu.ids gpurun_out/rot_*.log

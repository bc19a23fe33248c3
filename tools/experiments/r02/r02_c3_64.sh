#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
T="timeout -k 10 120 python tools/tune.py --rounds 6 --iters 20 --warm-ms 20"
$T --config c3 --len 64 --variants "default;WC_VARIANT=65536;WC_SHAPE=4,1,2;WC_SHAPE=4,1,2 WC_VARIANT=65536;WC_VARIANT=64;WC_SHAPE=4,2,2" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/c3_64.log

#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
T="timeout -k 10 120 python tools/tune.py --rounds 4 --iters 20 --warm-ms 20 --kind payload --headers"
echo "### c2 payload"; $T --config c2 --variants "default;WC_VARIANT=262144" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### slots 1500 +14 payload strided"; $T --config c3 --len 1500 --stride 2048 --offset 14 --variants "default;WC_VARIANT=262144" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### 256 +14 stride 2048 payload strided"; $T --config c3 --len 256 --stride 2048 --offset 14 --variants "default;WC_VARIANT=262144" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### c2 ip"; timeout -k 10 120 python tools/tune.py --rounds 4 --iters 20 --warm-ms 20 --config c2 2>&1 | grep -v amdgpu.ids || exit 1

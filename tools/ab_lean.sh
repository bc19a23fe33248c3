#!/usr/bin/env bash
# Lean kernel (aligned, one pass per packet) vs the previous paths
# (WC_LEAN_MAX=0: group kernel / seg kernel by the old table), C3 sizes,
# ip_cksum and payload_cksum over stamped UDP headers; then shapes for 64 B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
T="timeout -k 10 200 python tools/tune.py --rounds 7 --iters 40 --warm-ms 100"
for L in ${LENS:-64 128 256 512 768}; do
    echo "### $L ip"
    $T --config c3 --len $L --variants "default;WC_LEAN_MAX=0" 2>&1 | grep -v amdgpu.ids || exit 1
    echo "### $L payload"
    $T --config c3 --len $L --kind payload --headers --variants "default;WC_LEAN_MAX=0" 2>&1 | grep -v amdgpu.ids || exit 1
done
echo "### 256 shapes (ip / payload)"
$T --config c3 --len 256 --variants "default;WC_SHAPE=16,1,4;WC_SHAPE=8,2,4;WC_LEAN_MAX=0" 2>&1 | grep -v amdgpu.ids || exit 1
$T --config c3 --len 256 --kind payload --headers --variants "default;WC_SHAPE=16,1,4;WC_SHAPE=8,2,4;WC_LEAN_MAX=0" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### 64 ip shapes"
$T --config c3 --len 64 --variants "default;WC_SHAPE=4,1,2;WC_SHAPE=4,2,2;WC_SHAPE=8,1,4;WC_SHAPE=4,2,4;WC_SHAPE=8,1,8" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### 64 payload shapes"
$T --config c3 --len 64 --kind payload --headers --variants "default;WC_SHAPE=4,1,2;WC_SHAPE=8,1,4;WC_SHAPE=4,2,4" 2>&1 | grep -v amdgpu.ids || exit 1

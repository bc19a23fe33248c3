#!/usr/bin/env bash
# Small packets in 2048-B netmap slots at +14 (strided): ip_cksum vs
# payload_cksum over stamped UDP headers, per size.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
T="timeout -k 10 200 python tools/tune.py --rounds 5 --iters 40 --warm-ms 100"
for L in ${LENS:-64 128 256 1472}; do
    echo "### $L in 2048-B slots at +14: ip / payload"
    $T --config c3 --len $L --stride 2048 --offset 14 2>&1 | grep -v amdgpu.ids || exit 1
    $T --config c3 --len $L --stride 2048 --offset 14 --kind payload --headers 2>&1 | grep -v amdgpu.ids || exit 1
done

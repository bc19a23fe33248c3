#!/usr/bin/env bash
# Round 4: small payload_cksum in 2048-B slots at +14 -- ASIP (payload as
# ip_cksum over [8, len) + header terms; tuning build WC_VARIANT bit 27) on
# the narrow shapes, 64..240 B.  Rotating buffers (HBM).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
A=$((1 << 27))
T="timeout -k 10 200 python tools/tune.py --rounds 4 --iters 20 --rotate-bytes $((1 << 30))"
for L in 64 96 128 160 200 240; do
  V="default;WC_VARIANT=$A"
  for sh in 4,2,2 4,5,4 8,1,2 4,1,8 8,3,2; do
    V="$V;WC_SHAPE=$sh;WC_SHAPE=$sh WC_VARIANT=$A"
  done
  echo "== s14-$L payload+h"
  $T --config c3 --len $L --stride 2048 --offset 14 --kind payload --headers --variants "$V" \
    2>&1 | grep -v "^\s*round\|amdgpu.ids" || exit 1
  echo "== s14-$L ip"
  $T --config c3 --len $L --stride 2048 --offset 14 --variants "default" \
    2>&1 | grep -v "^\s*round\|amdgpu.ids" || exit 1
done

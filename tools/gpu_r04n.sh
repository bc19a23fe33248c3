#!/usr/bin/env bash
# Round 4 probe: what payload_cksum's header hand-off costs small packets in
# 2048-B slots (tuning build: WC_VARIANT bit 29 replaces it with constants --
# timing only, results wrong).  Rotating buffers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
P=$((1 << 29)); A=$((1 << 27))
T="timeout -k 10 200 python tools/tune.py --rounds 5 --iters 20 --rotate-bytes $((1 << 30))"
for L in 64 128; do
  echo "== s14-$L payload+h"
  $T --config c3 --len $L --stride 2048 --offset 14 --kind payload --headers \
    --variants "default;WC_VARIANT=$P;WC_VARIANT=$((P | A));WC_SHAPE=8,1,4 WC_VARIANT=$P" 2>&1 | grep -v "^\s*round\|amdgpu.ids" || exit 1
  echo "== s14-$L ip"
  $T --config c3 --len $L --stride 2048 --offset 14 --variants "default;WC_SHAPE=4,2,2" \
    2>&1 | grep -v "^\s*round\|amdgpu.ids" || exit 1
done

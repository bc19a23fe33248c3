#!/usr/bin/env bash
# Round 4: small payload_cksum packets in 2048-B slots at +14 (VERDICT r03
# item 6): header words from a direct load (HLOAD, WC_VARIANT bit 28) and/or
# payload as ip_cksum over [8, len) + header terms (ASIP, bit 27), per shape.
# Parity of the strided/payload GPU tests under both first.  Rotating buffers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
A=$((1 << 27)); H=$((1 << 28)); AH=$((A | H))
for v in $H $AH; do
  WC_TUNING=1 WC_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
      --timeout 120 --timeout-method thread -k "strided or payload" > gpurun_out/r04k_pytest_$v.log 2>&1 \
      || { tail -30 gpurun_out/r04k_pytest_$v.log; exit 1; }
  tail -1 gpurun_out/r04k_pytest_$v.log
done
T="timeout -k 10 200 python tools/tune.py --rounds 4 --iters 20 --rotate-bytes $((1 << 30))"
for L in 64 128 160 256; do
  V="default;WC_VARIANT=$H;WC_VARIANT=$AH"
  for sh in 8,1,4 4,2,2 8,2,4 8,3,2 4,2,4; do
    V="$V;WC_SHAPE=$sh WC_VARIANT=$H;WC_SHAPE=$sh WC_VARIANT=$AH"
  done
  echo "== s14-$L payload+h"
  $T --config c3 --len $L --stride 2048 --offset 14 --kind payload --headers --variants "$V" \
    2>&1 | grep -v "^\s*round\|amdgpu.ids" || exit 1
  echo "== s14-$L ip"
  $T --config c3 --len $L --stride 2048 --offset 14 --variants "default;WC_SHAPE=4,2,2;WC_SHAPE=8,1,4" \
    2>&1 | grep -v "^\s*round\|amdgpu.ids" || exit 1
done

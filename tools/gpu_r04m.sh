#!/usr/bin/env bash
# Round 4: planner change -- sparse payload_cksum of 7..16 chunks on (4,2,2).
# Parity (strided / payload / planner tests), then the new default against
# the previous shapes, and (4,2,2) on longer packets.  Rotating buffers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "strided or payload or planner" > gpurun_out/r04m_pytest.log 2>&1 \
    || { tail -30 gpurun_out/r04m_pytest.log; exit 1; }
tail -1 gpurun_out/r04m_pytest.log
T="timeout -k 10 200 python tools/tune.py --rounds 4 --iters 20 --rotate-bytes $((1 << 30))"
for L in 64 96 112 128 200 240; do
  echo "== s14-$L payload+h"
  $T --config c3 --len $L --stride 2048 --offset 14 --kind payload --headers \
    --variants "default;WC_SHAPE=8,1,4;WC_SHAPE=8,2,4" 2>&1 | grep -v "^\s*round\|amdgpu.ids" || exit 1
done
for L in 256 288 320 400 512; do
  echo "== s14-$L payload+h"
  $T --config c3 --len $L --stride 2048 --offset 14 --kind payload --headers \
    --variants "default;WC_SHAPE=4,2,2;WC_SHAPE=4,2,4;WC_SHAPE=8,2,4" 2>&1 | grep -v "^\s*round\|amdgpu.ids" || exit 1
  echo "== s14-$L ip"
  $T --config c3 --len $L --stride 2048 --offset 14 --variants "default;WC_SHAPE=4,2,2" \
    2>&1 | grep -v "^\s*round\|amdgpu.ids" || exit 1
done

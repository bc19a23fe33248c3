#!/usr/bin/env bash
# Round 4: payload_cksum header hand-off with a batch-uniform start phase
# (stride % 16 == 0): one DPP broadcast per window dword from a lane known
# per phase, instead of per-lane selects and two broadcasts.  Tuning build
# WC_VARIANT bit 30 = the previous per-lane hand-off.  Parity, then A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "strided or payload or planner or fused" > gpurun_out/r04o_pytest.log 2>&1 \
    || { tail -30 gpurun_out/r04o_pytest.log; exit 1; }
tail -1 gpurun_out/r04o_pytest.log
O=$((1 << 30))
T="timeout -k 10 200 python tools/tune.py --rounds 5 --iters 20 --rotate-bytes $((1 << 30))"
for L in 64 128 256; do
  echo "== s14-$L payload+h"
  $T --config c3 --len $L --stride 2048 --offset 14 --kind payload --headers \
    --variants "default;WC_VARIANT=$O;WC_SHAPE=8,1,4;WC_SHAPE=8,1,4 WC_VARIANT=$O" 2>&1 | grep -v "^\s*round\|amdgpu.ids" || exit 1
done
echo "== slot payload+h"
$T --config c3 --len 1500 --stride 2048 --offset 14 --kind payload --headers \
  --variants "default;WC_VARIANT=$O" 2>&1 | grep -v "^\s*round\|amdgpu.ids" || exit 1
echo "== c2 payload+h"
$T --config c2 --kind payload --headers --variants "default;WC_VARIANT=$O" 2>&1 | grep -v "^\s*round\|amdgpu.ids" || exit 1
echo "== c3-576 payload+h"
$T --config c3 --len 576 --offset 14 --stride 2048 --kind payload --headers --variants "default;WC_VARIANT=$O" 2>&1 | grep -v "^\s*round\|amdgpu.ids" || exit 1

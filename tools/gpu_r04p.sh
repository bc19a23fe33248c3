#!/usr/bin/env bash
# Round 4: the lean kernel's phase path (PH) for sparse packets at an even
# start phase (netmap slots at +14).  Parity first (the new lean-phase test
# and the strided / payload / planner tests), then PH against the group
# kernel (WC_LEAN_PHASE=0) and PH shapes.  Rotating buffers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "lean_phase or strided or payload or planner" > gpurun_out/r04p_pytest.log 2>&1 \
    || { tail -40 gpurun_out/r04p_pytest.log; exit 1; }
tail -1 gpurun_out/r04p_pytest.log
T="timeout -k 10 200 python tools/tune.py --rounds 4 --iters 20 --rotate-bytes $((1 << 30))"
for L in 64 128 256 576; do
  for k in ip payload; do
    h=""; [ $k = payload ] && h="--headers"
    echo "== s14-$L $k"
    $T --config c3 --len $L --stride 2048 --offset 14 --kind $k $h --variants \
      "default;WC_LEAN_PHASE=0;WC_SHAPE=4,1,4;WC_SHAPE=8,1,4;WC_SHAPE=8,1,8;WC_SHAPE=4,2,4;WC_SHAPE=8,2,4;WC_SHAPE=16,1,4;WC_SHAPE=8,3,2;WC_SHAPE=16,2,2;WC_SHAPE=16,3,1;WC_SHAPE=16,3,2" \
      2>&1 | grep -v "^\s*round\|amdgpu.ids" || exit 1
  done
done

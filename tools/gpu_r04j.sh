#!/usr/bin/env bash
# Round 4: small payload_cksum packets in 2048-B slots at +14 (VERDICT r03
# item 6).  payload_cksum as ip_cksum over [8, len) + per-packet header terms
# (ASIP, tuning build: WC_VARIANT bit 27) on every shape, against the
# header-range accumulate, per shape; ip_cksum alongside.  Rotating buffers
# (1 GiB of touched lines) so every launch reads HBM.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
A=$((1 << 27))
WC_TUNING=1 WC_VARIANT=$A timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -k "strided or payload" > gpurun_out/r04j_pytest.log 2>&1 \
    || { tail -30 gpurun_out/r04j_pytest.log; exit 1; }
tail -1 gpurun_out/r04j_pytest.log
T="timeout -k 10 200 python tools/tune.py --rounds 4 --iters 20 --rotate-bytes $((1 << 30))"
for L in 64 80 128 160 256; do
  echo "== s14-$L payload+h"
  $T --config c3 --len $L --stride 2048 --offset 14 --kind payload --headers --variants \
    "default;WC_VARIANT=$A;WC_SHAPE=8,1,4;WC_SHAPE=8,1,4 WC_VARIANT=$A;WC_SHAPE=8,2,4;WC_SHAPE=8,2,4 WC_VARIANT=$A;WC_SHAPE=8,3,2 WC_VARIANT=$A;WC_SHAPE=4,2,2 WC_VARIANT=$A" \
    2>&1 | grep -v "^\s*round\|amdgpu.ids" || exit 1
  echo "== s14-$L ip"
  $T --config c3 --len $L --stride 2048 --offset 14 --variants "default" 2>&1 | grep -v "^\s*round\|amdgpu.ids" || exit 1
done

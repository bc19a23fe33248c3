#!/usr/bin/env bash
# Round 4: deferred result stores in k_cksum_seg (WC_SEG_DEFER = tiles per
# wave).  Parity of the GPU parity suite with deferral forced on every
# seg-kernel launch, then A/B against the one-shot grid.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
WC_SEG_DEFER=8 WC_SEG_DEFER_MIN=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
    -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04i_pytest8.log 2>&1 \
    || { tail -30 gpurun_out/r04i_pytest8.log; exit 1; }
tail -1 gpurun_out/r04i_pytest8.log
WC_SEG_DEFER=3 WC_SEG_DEFER_MIN=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
    -m gpu -x -q --timeout 120 --timeout-method thread -k "ragged or seg or fused or zipf" \
    > gpurun_out/r04i_pytest3.log 2>&1 || { tail -30 gpurun_out/r04i_pytest3.log; exit 1; }
tail -1 gpurun_out/r04i_pytest3.log
CASES="c4:ip c4:payload+h c4:fused zslots:ip rslot:payload+h rc2:ip" \
VARS="default;WC_SEG_DEFER=8;WC_SEG_DEFER=4;WC_SEG_DEFER=2;WC_SEG_DEFER=8 WC_SEG_DEFER_MIN=1024" \
ROUNDS=3 bash tools/ab.sh

#!/bin/bash
# Round 2: whole-chunk flat tiles (edge bytes taken out per packet) vs the
# masked flat path -- parity of every ragged mode, then interleaved A/B.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "whole or zslots or walk" \
    --timeout 120 --timeout-method thread > gpurun_out/whole_pytest.log 2>&1 || { tail -30 gpurun_out/whole_pytest.log; exit 1; }
tail -3 gpurun_out/whole_pytest.log
T="timeout -k 10 200 python tools/tune.py --rounds 5 --iters 20"
V=${V:-"WC_WALK=0;WC_WALK=4096;WC_SEG=0;WC_SEG=0 WC_WALK=4096;WC_WALK=3 WC_GRP_ROWS=2"}
$T --config zslots --variants "$V" > gpurun_out/whole_zslots_ip.log 2>&1
$T --config zslots --kind payload --headers --variants "$V" > gpurun_out/whole_zslots_pl.log 2>&1
$T --config c4 --variants "WC_WALK=0;WC_WALK=4096;WC_SEG=0;WC_SEG=0 WC_WALK=4096" > gpurun_out/whole_c4.log 2>&1
$T --config c4 --kind payload --headers --variants "WC_WALK=0;WC_WALK=4096" > gpurun_out/whole_c4pl.log 2>&1
tail -n 7 gpurun_out/whole_*.log

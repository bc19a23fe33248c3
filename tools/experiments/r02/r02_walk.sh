#!/bin/bash
# Round 2: the walk path of k_cksum_seg -- parity of every ragged mode, then
# interleaved A/B against the flat / grouped / seg paths on zslots, netmap
# slots and C4.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "walk or zslots" \
    --timeout 120 --timeout-method thread > gpurun_out/walk_pytest.log 2>&1 || { tail -30 gpurun_out/walk_pytest.log; exit 1; }
tail -3 gpurun_out/walk_pytest.log
T="timeout -k 10 200 python tools/tune.py --rounds 5 --iters 20"
V=${V:-"WC_WALK=0;WC_WALK=2;WC_WALK=3;WC_WALK=2 WC_GRP_ROWS=2;WC_WALK=3 WC_GRP_ROWS=2"}
$T --config zslots --variants "$V" > gpurun_out/walk_zslots_ip.log 2>&1
$T --config zslots --kind payload --headers --variants "$V" > gpurun_out/walk_zslots_pl.log 2>&1
V2="WC_WALK=0;WC_WALK=$((2|0x300))"
$T --config c4 --variants "$V2" > gpurun_out/walk_c4.log 2>&1
$T --config c2 --ragged --offset 14 --stride 2048 --len 1500 --variants "$V2" > gpurun_out/walk_slots.log 2>&1
tail -n 8 gpurun_out/walk_*.log
exit 0
if [ -f tools/libwccksum_prev.so ]; then
    WC_LIB=tools/libwccksum_prev.so $T --config c4 > gpurun_out/walk_prev_c4.log 2>&1
    WC_LIB=tools/libwccksum_prev.so $T --config zslots > gpurun_out/walk_prev_zslots.log 2>&1
    $T --config c4 > gpurun_out/walk_new_c4.log 2>&1
    tail -n 2 gpurun_out/walk_prev_*.log gpurun_out/walk_new_c4.log
fi

#!/usr/bin/env bash
# Strided mid-size packets in 2048-B slots (no seg routing): planner shape vs
# candidates, aligned and at +14, tools/tune.py (one process per case).
export WC_NO_BUILD=1
V="default;WC_SHAPE=8,3,2;WC_SHAPE=8,2,4;WC_SHAPE=16,2,4;WC_SHAPE=8,1,4;WC_SHAPE=16,1,4;WC_SHAPE=16,3,4"
for L in 100 128 200 256 300 384 500; do
  for off in 0 14; do
    echo "== len $L +$off"
    timeout -k 10 120 python tools/tune.py --config c3 --len $L --stride 2048 --offset $off \
        --packets 1048576 --rounds 4 --iters 20 --variants "$V" 2>&1 | grep -v "round\|amdgpu" || exit 1
  done
done

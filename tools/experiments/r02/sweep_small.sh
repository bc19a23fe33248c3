#!/usr/bin/env bash
# Strided small / misaligned packets: group kernel shapes vs the seg kernel
# (WC_STRIDED_SEG=2) in one process per case (tools/tune.py).
export WC_NO_BUILD=1
T="timeout -k 10 120 python tools/tune.py --rounds 5 --iters 50"
run() { echo "== $1"; shift; $T "$@" > gpurun_out/sw.log 2>&1 || { tail gpurun_out/sw.log; exit 1; }; grep -v "round\|amdgpu" gpurun_out/sw.log; }
V="WC_STRIDED_SEG=0;WC_STRIDED_SEG=2"
run "64 aligned" --config c3 --len 64 --variants "$V;WC_STRIDED_SEG=0 WC_SHAPE=4,1,4"
run "64 +14" --config c3 --len 64 --offset 14 --variants "$V;WC_STRIDED_SEG=0 WC_SHAPE=4,2,2"
run "100 +0" --config c3 --len 100 --variants "$V"
run "256 +14" --config c3 --len 256 --offset 14 --variants "$V"
run "576 +14" --config c3 --len 576 --offset 14 --variants "$V"
run "1472 +14" --config c3 --len 1472 --offset 14 --variants "$V"
run "1472 +14 payload" --config c3 --len 1472 --offset 14 --kind payload --headers --variants "$V"
run "9000 +0" --config c3 --len 9000 --variants "$V"

#!/usr/bin/env bash
# Small packed packets (C3 64 B, 100 B, 144 B, 192 B) and the slot-stride effect (256 B at +14 in
# 2048 / 2304 / 2560-B slots).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
T="timeout -k 10 200 python tools/tune.py --rounds 4 --iters 20"
run() { local tag=$1; shift; echo "### $tag"; $T "$@" > gpurun_out/s2_$tag.log 2>&1 || { tail gpurun_out/s2_$tag.log; exit 1; }; grep -v "amdgpu.ids" gpurun_out/s2_$tag.log; }
run c3_64 --config c3 --len 64 --ceiling --variants "default;WC_SHAPE=4,1,2;WC_SHAPE=4,1,8;WC_SHAPE=4,1,16;WC_SHAPE=8,1,4;WC_SHAPE=8,1,8;WC_STRIDED_SEG=2 WC_VARIANT=2"
run len100 --config c3 --len 100 --variants "default;WC_SEG_ROWS=4;WC_STRIDED_SEG=0;WC_SEG_ROWS=8"
run len144 --config c3 --len 144 --variants "default;WC_VARIANT=2;WC_VARIANT=2 WC_SEG_ROWS=4;WC_SHAPE=4,5,4;WC_SHAPE=8,2,4"
run len192 --config c3 --len 192 --variants "default;WC_VARIANT=2;WC_VARIANT=2 WC_SEG_ROWS=4;WC_SHAPE=16,1,4"
for S in 2048 2304 2560 4096; do run slot256_$S --config c3 --len 256 --stride $S --offset 14; done

#!/usr/bin/env bash
# zslots: gathered path row-group sizes, and the slot-read ceiling of the ring's lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
T="timeout -k 10 200 python tools/tune.py --rounds 4 --iters 20"
$T --config zslots --ceiling --variants "default;WC_SEG_ROWS=2;WC_SEG_ROWS=8" > gpurun_out/zceil_ip.log 2>&1 || { tail gpurun_out/zceil_ip.log; exit 1; }
grep -v amdgpu.ids gpurun_out/zceil_ip.log
$T --config zslots --kind payload --headers --variants "default;WC_SEG_ROWS=2;WC_SEG_ROWS=8" > gpurun_out/zceil_pl.log 2>&1 || { tail gpurun_out/zceil_pl.log; exit 1; }
grep -v amdgpu.ids gpurun_out/zceil_pl.log
for L in 128 256; do
  $T --config c3 --len $L --stride 2048 --offset 14 > gpurun_out/zceil_s$L.log 2>&1 || { tail gpurun_out/zceil_s$L.log; exit 1; }
  echo "strided $L B in 2048-B slots at +14:"; grep -v amdgpu.ids gpurun_out/zceil_s$L.log
done

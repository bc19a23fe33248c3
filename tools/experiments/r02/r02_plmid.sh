#!/usr/bin/env bash
# payload_cksum, packed 576..1472 B: group kernel vs seg kernel (where does the seg path stop winning).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
T="timeout -k 10 120 python tools/tune.py --rounds 4 --iters 20 --warm-ms 20 --kind payload --headers"
out=gpurun_out/plm.log; : > $out
for off in 0 14; do
for L in 576 700 800 900 1024 1200 1400 1472; do
  echo "### c3 $L payload +$off (UDP headers)" | tee -a $out
  $T --config c3 --len $L --offset $off --variants "WC_STRIDED_SEG=0;WC_STRIDED_SEG=2 WC_SEG_ROWS=4;WC_STRIDED_SEG=2 WC_SEG_ROWS=8" 2>&1 | grep -v "amdgpu.ids" | tee -a $out || exit 1
done
done

#!/usr/bin/env bash
# payload_cksum on small packed packets: group kernel vs seg kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
T="timeout -k 10 120 python tools/tune.py --rounds 4 --iters 20 --warm-ms 20 --kind payload --headers"
out=gpurun_out/pls.log; : > $out
for L in 64 100 128 144 192 256 320 400 576; do
  echo "### c3 $L payload (UDP headers)" | tee -a $out
  $T --config c3 --len $L --variants "default;WC_STRIDED_SEG=0;WC_STRIDED_SEG=2 WC_SEG_ROWS=2;WC_STRIDED_SEG=2 WC_SEG_ROWS=4" 2>&1 | grep -v "amdgpu.ids" | tee -a $out || exit 1
done
for L in 64 256; do
  echo "### c3 $L payload +14 (UDP headers)" | tee -a $out
  $T --config c3 --len $L --offset 14 --variants "default;WC_STRIDED_SEG=0;WC_STRIDED_SEG=2 WC_SEG_ROWS=2;WC_STRIDED_SEG=2 WC_SEG_ROWS=4" 2>&1 | grep -v "amdgpu.ids" | tee -a $out || exit 1
done

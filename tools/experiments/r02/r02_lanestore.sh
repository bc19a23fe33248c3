#!/usr/bin/env bash
# Coalesced result store (lane j = packet p0 + j) in the strided kernel, and the
# aligned-small planner change: parity, then A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/ls_pytest.log 2>&1 || { tail -40 gpurun_out/ls_pytest.log; exit 1; }
tail -1 gpurun_out/ls_pytest.log
T="timeout -k 10 120 python tools/tune.py --rounds 5 --iters 20 --warm-ms 20"
out=gpurun_out/ls.log; : > $out
for L in 64 80 144 256 576 1472; do
  echo "### c3 $L" | tee -a $out
  $T --config c3 --len $L --variants "WC_VARIANT=128;default;WC_VARIANT=64" 2>&1 | grep -v "amdgpu.ids" | tee -a $out || exit 1
done
for L in 64 256; do
  echo "### c3 $L payload" | tee -a $out
  $T --config c3 --len $L --kind payload --headers --variants "WC_VARIANT=128;default" 2>&1 | grep -v "amdgpu.ids" | tee -a $out || exit 1
done
echo "### slots 1500 +14 ragged small batch (group kernel path n/a) / c2" | tee -a $out
$T --config c2 --variants "WC_VARIANT=128;default" 2>&1 | grep -v "amdgpu.ids" | tee -a $out || exit 1

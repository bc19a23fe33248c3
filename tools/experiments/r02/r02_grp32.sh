#!/bin/bash
# Grouped path with 32 lanes per packet: ragged parity, then A/B on netmap
# slot rings (ragged) of several sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ragged or grp or slot or dense or host or fused" --timeout 240 --timeout-method thread \
    > gpurun_out/grp32_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/grp32_pytest.log
[ $rc -eq 0 ] || exit $rc
T="timeout -k 10 200 python tools/tune.py --rounds 4 --iters 20"
V="WC_GRP_PW32=255;default;WC_GRP_PW32=0;WC_GRP_PW32=48"
for L in 1500 1200 1000 800 600; do
  echo "## ragged slots len $L ip"; $T --config c3 --len $L --stride 2048 --offset 14 --ragged --variants "$V" 2>&1 | grep -v amdgpu.ids
  echo "## ragged slots len $L payload+h"; $T --config c3 --len $L --stride 2048 --offset 14 --ragged --kind payload --headers --variants "$V" 2>&1 | grep -v amdgpu.ids
done
echo "## zslots"; $T --config zslots --variants "WC_GRP_PW32=255;default" 2>&1 | grep -v amdgpu.ids
echo "## c4"; $T --config c4 --variants "WC_GRP_PW32=255;default" 2>&1 | grep -v amdgpu.ids

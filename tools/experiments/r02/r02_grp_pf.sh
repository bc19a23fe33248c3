#!/bin/bash
# Grouped path with prefetched unit descriptors: ragged parity, then A/B vs
# the previous build on netmap slot rings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ragged or grp or slot or dense or host or fused" --timeout 240 --timeout-method thread \
    > gpurun_out/grppf_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/grppf_pytest.log
[ $rc -eq 0 ] || exit $rc
T="timeout -k 10 200 python tools/tune.py --rounds 4 --iters 20"
for a in "--config c3 --len 1500 --stride 2048 --offset 14 --ragged" "--config c3 --len 1500 --stride 2048 --offset 14 --ragged --kind payload --headers" "--config c3 --len 1000 --stride 2048 --offset 14 --ragged"; do
  for rep in 1 2; do
    echo -n "prev $a: "; WC_LIB=tools/libwccksum_prev.so $T $a 2>&1 | grep -v amdgpu.ids
    echo -n "new  $a: "; $T $a --variants "default;WC_GRP_PW32=0" 2>&1 | grep -v amdgpu.ids | tr '\n' '|'; echo
  done
done

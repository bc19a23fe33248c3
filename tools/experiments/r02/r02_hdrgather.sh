#!/usr/bin/env bash
# Fused IPv4 header + payload ragged pass (k_cksum_seg HDR): gathered path compiled in (new) vs flat fallback only (prev).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fused or ip_udp or header or ragged or zslots" \
    > gpurun_out/hg_pytest.log 2>&1 || { tail -40 gpurun_out/hg_pytest.log; exit 1; }
tail -1 gpurun_out/hg_pytest.log
T="timeout -k 10 120 python tools/tune.py --rounds 3 --iters 20 --warm-ms 20 --kind payload --headers --fused"
for c in "zslots" "c4" "c3 --len 1500 --stride 2048 --offset 14 --ragged"; do
  for rep in 1 2; do
    echo -n "prev $c: "; WC_LIB=tools/libwccksum_prev.so $T --config $c 2>&1 | grep -v amdgpu.ids || exit 1
    echo -n "new  $c: "; $T --config $c 2>&1 | grep -v amdgpu.ids || exit 1
  done
done

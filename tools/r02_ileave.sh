#!/usr/bin/env bash
# Block-interleaved sparse tiles (WC_VARIANT bit 20): parity of the ragged tests with it on, then A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
WC_VARIANT=1048576 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ragged or zslots or golden or slot or c4 or host or linux or verify or fused or ip_udp" \
    > gpurun_out/il_pytest.log 2>&1 || { tail -40 gpurun_out/il_pytest.log; exit 1; }
tail -1 gpurun_out/il_pytest.log
CASES="rslot:ip rslot:payload+h zslots:ip zslots:payload+h c4:ip c4r:ip" VARS="default;WC_VARIANT=1048576" ROUNDS=4 bash tools/ab.sh

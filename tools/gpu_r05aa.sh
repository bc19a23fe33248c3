#!/usr/bin/env bash
# Round 5, call aa / af: RX parse changes -- RX parity in every mode, then the rings timed.
# windows (half the VALU of per-chunk byte masks) -- RX parity in every mode,
# then the rings timed (compare call y's defaults: 112.8 / 97.1 / 236.3 us).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05aa}
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rx.py \
    > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
T="timeout -k 10 300 python tools/tune.py --rounds 4 --iters 200"
$T --config zrx > $OUT/zrx.log 2>&1 || exit 1
$T --config zrx --rx-arp 3 > $OUT/zrx3.log 2>&1 || exit 1
$T --config rx --iters 100 > $OUT/rx.log 2>&1 || exit 1
for f in zrx zrx3 rx; do grep -E "^default" $OUT/$f.log; done

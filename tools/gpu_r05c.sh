#!/usr/bin/env bash
# Round 5, call c: the resident server's cost to a concurrent C2 batch
# (none / idle / busy), and the C host-latency table with the persistent
# 16-thread CPU pool (profiles/host_latency_r05.log).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R05C_OUT:-r05c}
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 300 python -u tools/serve_interference.py --rounds 5 > $OUT/serve_interference.log 2>&1
rc=$?; tail -6 $OUT/serve_interference.log; [ $rc -eq 0 ] || exit $rc
python3 -c "import sys; sys.path.insert(0, 'tests'); from cprog import build; build('host_latency', '$OUT')" \
    > $OUT/build.log 2>&1 || { cat $OUT/build.log; exit 1; }
timeout -k 10 400 $OUT/host_latency 16 0.4 > $OUT/host_latency.log 2>&1
rc=$?; tail -3 $OUT/host_latency.log; exit $rc

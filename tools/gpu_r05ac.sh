#!/usr/bin/env bash
# Round 5, call ac: round measurements of the RX rings with the final RX
# kernel (header-sum change): bench lines, rocprof kernel stats, FETCH_SIZE /
# WRITE_SIZE passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFGS="zrx zrxa3 rx" TAG=r05f bash tools/round_measure.sh > gpurun_out/round_r05f.log 2>&1
rc=$?; grep -E "^==|rc=" gpurun_out/round_r05f.log | tail -20; exit $rc

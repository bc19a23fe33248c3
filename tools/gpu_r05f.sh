#!/usr/bin/env bash
# Round 5, call f: bench lines + rocprofv3 kernel stats / FETCH_SIZE /
# WRITE_SIZE (separate passes) for the round's changed paths: C2 (headline),
# C5 (split launches), the RX rings under ADAPT (all-UDP, every third ARP,
# MTU), C4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFGS="${CFGS:-c2 c5 zrx zrxa3 rx c4}" TAG=${TAG:-r05} bash tools/round_measure.sh \
    > gpurun_out/round_r05.log 2>&1
rc=$?; grep -E "^==|rc=" gpurun_out/round_r05.log | tail -30; exit $rc

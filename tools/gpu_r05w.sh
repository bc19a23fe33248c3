#!/usr/bin/env bash
# Round 5, call w: dynamic instruction counts (rocprofv3 --pmc, one counter
# group per run) of the RX verdict kernel on the mixed ring, the plain ragged
# payload_cksum on the same slots, and C4 -- where the issue-bound half of
# the mixed ring's time goes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp WC_NO_BUILD=1
TAG=zrx TUNE_ARGS="--config zrx --rounds 1 --iters 5 --warm-ms 5" bash tools/pmc_ab.sh || exit 1
TAG=zsl TUNE_ARGS="--config zslots --kind payload --headers --rounds 1 --iters 5 --warm-ms 5" bash tools/pmc_ab.sh || exit 1
TAG=c4 TUNE_ARGS="--config c4 --rounds 1 --iters 3 --warm-ms 5" bash tools/pmc_ab.sh || exit 1

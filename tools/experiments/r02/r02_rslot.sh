#!/usr/bin/env bash
# Ragged 1500-B netmap ring: grouped path vs gathered path; C4: seg vs gathered.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
CASES="rslot:ip rslot:payload+h c4:ip" VARS="default;WC_GRP_SPARSE=65;WC_GRP_SPARSE=65 WC_GATHER=2" ROUNDS=4 bash tools/ab.sh

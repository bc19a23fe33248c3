#!/usr/bin/env bash
# XCD remap super-block span (WC_VARIANT bits 8..15 = log2 span; 0 = 4096 workgroups) on the seg kernel configs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
CASES="c4:ip rslot:ip zslots:ip c3-300:ip" VARS="default;WC_VARIANT=2560;WC_VARIANT=2816;WC_VARIANT=3328;WC_VARIANT=3584;WC_VARIANT=8" ROUNDS=3 bash tools/ab.sh

#!/bin/bash
# PMC instruction mix of the ragged paths on the mixed-size netmap ring.
set -e
export WC_NO_BUILD=1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=zflat TUNE_ARGS="--config zslots --rounds 1 --iters 3 --variants WC_SEG=0" bash tools/pmc.sh
TAG=zgrp TUNE_ARGS="--config zslots --rounds 1 --iters 3 --variants default" bash tools/pmc.sh
TAG=zsegflat TUNE_ARGS="--config zslots --rounds 1 --iters 3 --variants WC_GRP_SPARSE=65" bash tools/pmc.sh

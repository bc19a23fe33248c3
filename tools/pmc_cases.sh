#!/usr/bin/env bash
# tools/pmc_ab.sh over a list of cases, one TAG each:
#   CASES="c4pl:--config c4 --kind payload --headers|c4f:--config c4 --fused --headers"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
IFS='|' read -ra list <<< "$CASES"
for c in "${list[@]}"; do
    tag=${c%%:*}; args=${c#*:}
    echo "=== $tag: $args"
    TAG=$tag TUNE_ARGS="$args --rounds 1 --iters 3" bash tools/pmc_ab.sh || exit 1
done

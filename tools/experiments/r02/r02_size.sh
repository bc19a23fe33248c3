#!/bin/bash
# Batch-size dependence of the ragged (seg, grouped path) vs strided group
# kernel on 1500-B netmap slots at +14.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
T="timeout -k 10 200 python tools/tune.py --rounds 3 --iters 10"
for P in 262144 1048576 4194304; do
  echo "## $P packets ragged"; $T --config c3 --len 1500 --stride 2048 --offset 14 --ragged --packets $P 2>&1 | grep -v amdgpu.ids
  echo "## $P packets strided"; $T --config c3 --len 1500 --stride 2048 --offset 14 --packets $P 2>&1 | grep -v amdgpu.ids
done

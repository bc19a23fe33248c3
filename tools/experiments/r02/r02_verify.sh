#!/bin/bash
# Full GPU parity suite, the default bench line, and the C3 sizes + slots
# through tune.py (new planner).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/verify_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/verify_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/verify_bench.json 2> gpurun_out/verify_bench.err || exit 1
cat gpurun_out/verify_bench.json
T="timeout -k 10 200 python tools/tune.py --rounds 4 --iters 20"
for a in "--config c2" "--config c2 --kind payload --headers" "--config c3 --len 1024" "--config c3 --len 1500 --stride 2048 --offset 14" "--config c3 --len 800"; do
  echo "## $a"; $T $a 2>&1 | grep -v amdgpu.ids
done

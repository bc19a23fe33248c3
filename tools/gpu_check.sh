#!/usr/bin/env bash
# GPU-box check sequence: smoke -> gpu parity tests -> 1-GPU bench.
# Each GPU step has its own time limit; a fault / abort / timeout stops the
# script (only an ordinary test failure, exit 1, lets the bench still run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

stop_if_fault() {  # $1 = exit code, $2 = step
    case "$1" in
        0|1) return 0 ;;
        *) echo "step $2 ended with $1: stopping" | tee -a "$OUT/summary.log"; exit "$1" ;;
    esac
}

echo "== smoke" | tee "$OUT/summary.log"
timeout -k 10 420 python -c "import __graft_entry__ as g; g.build(); g.smoke(); \
print('loaded:', sorted({l.split()[-1] for l in open('/proc/self/maps') if 'wccksum' in l}))" \
    > "$OUT/smoke.log" 2>&1
rc=$?; tail -4 "$OUT/smoke.log" | tee -a "$OUT/summary.log"; stop_if_fault $rc smoke
git_sha=$(cat .head_sha 2>/dev/null || echo unknown); echo "tree: $git_sha" | tee -a "$OUT/summary.log"

echo "== pytest -m gpu" | tee -a "$OUT/summary.log"
timeout -k 10 900 python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -15 "$OUT/pytest_gpu.log" | tee -a "$OUT/summary.log"; stop_if_fault $rc pytest

echo "== bench" | tee -a "$OUT/summary.log"
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
rc=$?; tail -2 "$OUT/bench.log" | tee -a "$OUT/summary.log"; stop_if_fault $rc bench
exit 0

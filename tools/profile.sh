#!/usr/bin/env bash
# rocprofv3 passes over the 1-GPU bench (run on the GPU box):
#   1. --kernel-trace --stats          (per-kernel durations)
#   2. --pmc FETCH_SIZE  (own pass)    (HBM read bytes; x2 on gfx950, see guide)
#   3. --pmc WRITE_SIZE  (own pass)
# Output under gpurun_out/prof_<tag>/.  BENCH_ARGS selects the workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$PWD
TAG=${TAG:-r01}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---steps 50 --warmup 5 --no-cpu-baseline --no-c5 --no-extra}

run() {  # $1 = name, rest = rocprofv3 options
    local name=$1; shift
    (cd /tmp && timeout -k 10 600 rocprofv3 "$@" -d "$OUT/$name" -o run \
        --output-format csv -- python3 "$REPO/bench.py" $ARGS) > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a "$OUT/summary.log"
    case $rc in 0) ;; *) exit $rc ;; esac
    # keep gpurun_out/ small (it travels back, <= 64 MiB): the per-dispatch
    # trace is summarised by run_kernel_stats.csv; counters are compressed
    rm -f "$OUT/$name/run_kernel_trace.csv"
    [ -f "$OUT/$name/run_counter_collection.csv" ] && gzip -f "$OUT/$name/run_counter_collection.csv"
    return 0
}

run stats --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
exit 0

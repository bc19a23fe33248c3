#!/usr/bin/env bash
# One GPU call as a list of named steps (run on the GPU box through gpurun).
# Replaces the per-call tools/gpu_rNN*.sh scripts of earlier rounds.
#
#   TAG=r06a STEPS="pytest smoke bench prof_c2" bash tools/gpu_steps.sh
#
# Every step has its own time limit and writes under gpurun_out/$TAG/; the
# first step that fails (test failure, fault, abort, time limit) ends the
# call -- nothing else touches the GPU after it.
#   pytest        the whole -m gpu suite (PYTEST_ARGS adds options / a -k filter)
#   smoke         __graft_entry__.smoke()
#   bench         the driver's command: bench.py --gpus 1 --steps 20 --warmup 5
#   bench_args    bench.py $BENCH_ARGS (> bench_args.json)
#   prof_c2       rocprofv3 --kernel-trace --stats of the driver's headline command
#   diag_headline tools/diag_headline.py (the headline's whole-job gap, by issue mode)
#   tune          tools/tune.py once per '|'-separated argument set in $TUNE_ARGS
#                 (> tune1.log, tune2.log, ...; quote --variants specs inside)
#   e2e           tools/e2e.py $E2E_ARGS (host-path variants, end to end)
#   ab            A/B of WC_LIB=$AB_LIB against the in-tree library, tune.py $AB_ARGS
#                 (';'-separated cases), $AB_REPS alternating rounds
#   round         tools/round_measure.sh with CFGS (bench line + rocprof + PMC passes)
#   pmc           one rocprofv3 --pmc pass per counter group in PMC_GROUPS ("A B;C D")
#                 over bench.py $PMC_BENCH_ARGS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$PWD
TAG=${TAG:-r06}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp WC_NO_BUILD=1

step() {  # $1 = name, $2 = seconds, rest = command; stdout/stderr -> $OUT/$1.log
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    local t0=$SECONDS
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -4 "$OUT/$name.log"
    echo "$name rc=$rc wall_s=$((SECONDS - t0))" >> "$OUT/summary.log"
    if [ $rc -ne 0 ]; then
        echo "step $name ended with $rc: stopping"
        exit $rc
    fi
}

for s in ${STEPS:-pytest smoke bench}; do
    case $s in
        pytest)
            step pytest 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 \
                --timeout-method thread ${PYTEST_ARGS:-} ;;
        smoke)
            step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
        bench)
            step bench 600 python bench.py --gpus 1 --steps 20 --warmup 5
            grep '^{' "$OUT/bench.log" > "$OUT/bench.json" ;;
        bench_args)
            step bench_args 600 python bench.py ${BENCH_ARGS:-}
            grep '^{' "$OUT/bench_args.log" > "$OUT/bench_args.json" ;;
        prof_c2)
            (cd /tmp && step prof_c2 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run \
                --output-format csv -- python3 "$REPO/bench.py" --gpus 1 --steps 20 --warmup 5 \
                --no-c5 --no-extra --no-e2e --no-cpu-baseline) || exit $?
            rm -f "$OUT/prof_c2/run_kernel_trace.csv"
            head -4 "$OUT/prof_c2/run_kernel_stats.csv" ;;
        diag_headline)
            step diag_headline 300 python tools/diag_headline.py --json "$OUT/diag_headline.json" ;;
        tune)
            IFS='|' read -ra runs <<< "${TUNE_ARGS:-}"
            k=0
            for a in "${runs[@]}"; do
                k=$((k + 1))
                eval "step tune$k 600 python tools/tune.py $a"
            done ;;
        e2e)
            step e2e 500 python tools/e2e.py ${E2E_ARGS:-} ;;
        ab)
            # A/B of two builds in alternating fresh processes: WC_LIB=$AB_LIB
            # (A) against the in-tree product library (B), tune.py $AB_ARGS
            # for each ';'-separated case, $AB_REPS times.
            IFS=';' read -ra cases <<< "${AB_ARGS:---config zrx}"
            for rep in $(seq 1 "${AB_REPS:-3}"); do
                c=0
                for a in "${cases[@]}"; do
                    c=$((c + 1))
                    step ab_A${c}_$rep 200 env WC_TUNING=0 WC_LIB="$AB_LIB" python tools/tune.py $a --rounds 3 --iters 20
                    step ab_B${c}_$rep 200 env WC_TUNING=0 WC_LIB="$REPO/warpcore_amd/libwccksum.so" python tools/tune.py $a --rounds 3 --iters 20
                done
            done ;;
        round)
            step round 1200 env TAG="$TAG" CFGS="${CFGS:-c2}" bash tools/round_measure.sh ;;
        pmc)
            IFS=';' read -ra groups <<< "${PMC_GROUPS:-FETCH_SIZE;WRITE_SIZE}"
            k=0
            for g in "${groups[@]}"; do
                k=$((k + 1))
                (cd /tmp && step pmc$k 120 rocprofv3 --pmc $g -d "$OUT/pmc$k" -o run \
                    --output-format csv -- python3 "$REPO/bench.py" ${PMC_BENCH_ARGS:---no-extra --no-c5 --no-e2e --no-cpu-baseline --steps 20}) || exit $?
                [ -f "$OUT/pmc$k/run_counter_collection.csv" ] && gzip -f "$OUT/pmc$k/run_counter_collection.csv"
            done ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
exit 0

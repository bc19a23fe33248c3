#!/usr/bin/env bash
# One GPU call's worth of round-end measurements (run on the GPU box):
# bench lines (with CPU baseline) and rocprofv3 passes (kernel stats,
# FETCH_SIZE, WRITE_SIZE -- separate runs) for the configs in CFGS.
#   CFGS="c2 c4 c4pl slotspl"  TAG=r01
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
TAG=${TAG:-r02}
mkdir -p gpurun_out/round
for c in ${CFGS:-c2 c4 c4pl slotspl}; do
    case $c in
        c2) a="--config c2" ;;
        c2pl) a="--config c2 --kind payload --headers" ;;
        c4) a="--config c4" ;;
        c4pl) a="--config c4 --kind payload --headers" ;;
        c4plr) a="--config c4 --kind payload" ;;
        slots) a="--config slots" ;;
        slotspl) a="--config slots --kind payload --headers" ;;
        c5) a="--config c5" ;;
        c3_*) a="--config c3 --len ${c#c3_}" ;;
        zslots) a="--config zslots" ;;
        zslotspl) a="--config zslots --kind payload --headers" ;;
        c2f) a="--config c2 --fused" ;;
        c4f) a="--config c4 --fused" ;;
        slotsf) a="--config slots --fused" ;;
        zslotsf) a="--config zslots --fused" ;;
        rx) a="--config rx" ;;
        zrx) a="--config zrx" ;;
        zrxa3) a="--config zrx --rx-arp 3" ;;
        c3pl_*) a="--config c3 --len ${c#c3pl_} --kind payload --headers" ;;
        s14_*) a="--config c3 --len ${c#s14_} --stride 2048 --offset 14" ;;
        s14pl_*) a="--config c3 --len ${c#s14pl_} --stride 2048 --offset 14 --kind payload --headers" ;;
        *) echo "unknown config $c"; exit 2 ;;
    esac
    echo "== $c: bench"
    c5=""; [ "$c" = c2 ] || c5="--no-c5"   # the C5 leg rides on the headline line
    timeout -k 10 300 python bench.py $a $c5 > gpurun_out/round/bench_${TAG}_$c.json \
        2> gpurun_out/round/bench_${TAG}_$c.err || { tail gpurun_out/round/bench_${TAG}_$c.err; exit 1; }
    cat gpurun_out/round/bench_${TAG}_$c.json
    echo "== $c: rocprof"
    TAG=${TAG}_$c BENCH_ARGS="$a --steps 50 --warmup 5 --no-cpu-baseline --no-c5 --no-extra --no-e2e --graph off" tools/profile.sh || exit 1
done

#!/usr/bin/env bash
# the C5 window (2^25 x 1472 B = 49 GB in one launch)
# against C2 (2^20) on the same kernel.  (1) HIP-event timing over window
# sizes and allocators (torch / hipMalloc / contiguous), (2) XCD super-block
# spans (tuning build), (3) rocprofv3 --pmc passes -- address translation
# (UTCL1/UTCL2), EA read requests, wave waiting -- one counter group per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$PWD
OUT=$REPO/gpurun_out/c5probe${TAG:+_$TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp WC_NO_BUILD=1

if [ -z "${SKIP_TIMING:-}" ]; then
timeout -k 10 300 python3 -u tools/c5_window.py --windows 1048576,4194304,8388608,33554432 \
    --allocs torch,hip,contig --rounds 3 > "$OUT/timing.log" 2>&1 \
    || { tail -20 "$OUT/timing.log"; exit 1; }
tail -14 "$OUT/timing.log"
timeout -k 10 300 python3 -u tools/c5_window.py --windows 1048576,33554432 --allocs torch \
    --variants "default;WC_VARIANT=2560;WC_VARIANT=2816;WC_VARIANT=3584;WC_VARIANT=4096;WC_VARIANT=7936" \
    --rounds 3 > "$OUT/spans.log" 2>&1 || { tail -20 "$OUT/spans.log"; exit 1; }
tail -13 "$OUT/spans.log"
fi

pass() {  # $1 = case name, $2 = tool args, $3 = pass name, rest = counters
    local c=$1 targs=$2 name=$3; shift 3
    mkdir -p "$OUT/$c"
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$c/$name" -o run \
        --output-format csv -- python3 "$REPO/tools/c5_window.py" $targs --rounds 1 --iters 3 \
        --warm-ms 0) > "$OUT/$c/$name.log" 2>&1
    local rc=$?
    echo "$c $name rc=$rc" | tee -a "$OUT/summary.log"
    [ $rc -eq 0 ] || { tail -5 "$OUT/$c/$name.log"; exit $rc; }
}
for c in c2 c5 c5contig; do
    case $c in
        c2) t="--windows 1048576 --allocs torch" ;;
        c5) t="--windows 33554432 --allocs torch" ;;
        c5contig) t="--windows 33554432 --allocs contig" ;;
    esac
    pass $c "$t" utcl1 TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_PERMISSION_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE
    pass $c "$t" utcl1s TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum
    pass $c "$t" ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_BUSY_avr
    pass $c "$t" sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
    for f in "$OUT/$c"/*/run_counter_collection.csv; do gzip -kf "$f"; done
    python3 tools/pmc_report.py "$OUT/$c" > "$OUT/$c/report.txt" 2>&1
    cat "$OUT/$c/report.txt"
done
exit 0

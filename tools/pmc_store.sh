#!/usr/bin/env bash
# Round 4: why do C4's result writes cost more than
# their bandwidth time?  The seg kernel on C4 with and without its result
# store (tuning build, WC_VARIANT bit 24), one rocprofv3 --pmc pass per
# counter group, counters only.  CASE picks the workload (tune.py args).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$PWD
OUT=$REPO/gpurun_out/pmc_store${TAG:+_$TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp WC_NO_BUILD=1 WC_TUNING=1
CASE=${CASE:---config c4}
pass() {  # $1 = variant name, $2 = WC_VARIANT, $3 = pass name, rest = counters
    local v=$1 var=$2 name=$3; shift 3
    (cd /tmp && WC_VARIANT=$var timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$v/$name" -o run \
        --output-format csv -- python3 "$REPO/tools/tune.py" $CASE --rounds 1 --iters 5 --warm-ms 5) \
        > "$OUT/$v/$name.log" 2>&1
    local rc=$?
    echo "$v $name rc=$rc" | tee -a "$OUT/summary.log"
    [ $rc -eq 0 ] || { tail -5 "$OUT/$v/$name.log"; exit $rc; }
}
for v in store nostore; do
    var=0; [ $v = nostore ] && var=16777216
    mkdir -p "$OUT/$v"
    pass $v $var ea_wr TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum
    pass $v $var ea_rd TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_WRITEBACK_sum
    pass $v $var ea_lvl TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_LEVEL_sum TCC_WRITE_sum TCC_HIT_sum
    pass $v $var sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
    pass $v $var ta TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_MISS_sum TCC_REQ_sum
    python3 tools/pmc_report.py "$OUT/$v" > "$OUT/$v/report.txt"
    cat "$OUT/$v/report.txt"
done

#!/usr/bin/env bash
# PMC passes over tools/tune.py A/B variants (one rocprofv3 run per counter
# group, counters only).  TAG, TUNE_ARGS as in pmc.sh.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$PWD
TAG=${TAG:-x}
OUT=$REPO/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp WC_NO_BUILD=1
ARGS=${TUNE_ARGS:---config c4 --rounds 1 --iters 3}
pass() {
    local name=$1; shift
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run \
        --output-format csv -- python3 "$REPO/tools/tune.py" $ARGS) > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a "$OUT/summary.log"
    case $rc in 0) ;; *) tail -5 "$OUT/$name.log"; exit $rc ;; esac
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD
pass sq2 SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE
pass tcc FETCH_SIZE
pass tcc2 TCC_HIT_sum TCC_MISS_sum
${EXTRA_PASS:+pass extra $EXTRA_PASS}
python3 tools/pmc_report.py "$OUT"

#!/usr/bin/env bash
# PMC passes (one rocprofv3 run per counter group; no trace domains mixed in)
# over tools/tune.py with TUNE_ARGS.  Output: gpurun_out/pmc_<TAG>/<pass>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$PWD
TAG=${TAG:-x}
OUT=$REPO/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${TUNE_ARGS:---config c4 --rounds 1 --iters 3}

pass() {  # $1 = name, rest = counters
    local name=$1; shift
    (cd /tmp && timeout -k 10 300 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run \
        --output-format csv -- python3 "$REPO/tools/tune.py" $ARGS) > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a "$OUT/summary.log"
    case $rc in 0) ;; *) exit $rc ;; esac
}

pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
pass sq2 SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE
pass tcc FETCH_SIZE
exit 0

#!/bin/bash
# Memory-pipeline PMC passes (TA / TCP / SQ) for C2 strided, the ragged
# 1500-B slot ring (grouped path) and the mixed-size ring (flat path).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$PWD
export WC_NO_BUILD=1 TMPDIR=/tmp
pass() {  # $1 tag $2 name, rest counters; TUNE_ARGS from env
    local tag=$1 name=$2; shift 2
    local out=$REPO/gpurun_out/pmcd_$tag
    mkdir -p $out
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$out/$name" -o run --output-format csv -- \
        python3 "$REPO/tools/tune.py" $TUNE_ARGS) > "$out/$name.log" 2>&1
    echo "$tag $name rc=$?"
}
for w in "c2|--config c2 --rounds 1 --iters 3" "rslot|--config c3 --len 1500 --stride 2048 --offset 14 --ragged --rounds 1 --iters 3" "zslots|--config zslots --rounds 1 --iters 3"; do
  tag=${w%%|*}; TUNE_ARGS=${w#*|}
  pass $tag tcp TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum || exit 1
  pass $tag ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL || exit 1
  pass $tag tcp2 TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_LATENCY_sum || exit 1
  python3 tools/pmc_report.py gpurun_out/pmcd_$tag > gpurun_out/pmcd_$tag.txt
done
cat gpurun_out/pmcd_*.txt | grep -v "copyBuffer" 

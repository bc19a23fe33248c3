#!/bin/bash
# PMC instruction mix / waits of the walk path vs the flat path (zslots).
set -e
export WC_NO_BUILD=1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=zflat TUNE_ARGS="--config zslots --rounds 1 --iters 3 --variants WC_WALK=0" bash tools/pmc.sh
TAG=zwalk4 TUNE_ARGS="--config zslots --rounds 1 --iters 3 --variants WC_WALK=2" bash tools/pmc.sh
python3 tools/pmc_report.py gpurun_out/pmc_zflat > gpurun_out/pmc_zflat.txt
python3 tools/pmc_report.py gpurun_out/pmc_zwalk4 > gpurun_out/pmc_zwalk4.txt
cd /tmp && timeout -k 10 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d $GRAFT_REPO_ROOT/gpurun_out/pmc_tcp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/tune.py --config zslots --rounds 1 --iters 3 --variants "WC_WALK=0;WC_WALK=2" > $GRAFT_REPO_ROOT/gpurun_out/pmc_tcp.log 2>&1 || true

#!/usr/bin/env bash
# Round 5, call z (closing check on the final tree): the whole GPU suite,
# smoke(), the driver's bench command, and rocprofv3 kernel stats of the
# driver's command (C2 kernel average vs the line's kernel_ms_avg).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$PWD
OUT=$REPO/gpurun_out/${TAG:-r05z}
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > $OUT/smoke.log 2>&1
rc=$?; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err \
    || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/bench.json'))
r = d['roofline']; print('C2', d['value'], r['frac'], r['frac_job'], r['kernel_ms_avg'], 'C5', d['c5']['frac_kernel'])"
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
    -- python3 $REPO/bench.py --gpus 1 --steps 20 --warmup 5 --no-c5 --no-extra --no-cpu-baseline) \
    > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
rm -f $OUT/prof/run_kernel_trace.csv
head -5 $OUT/prof/run_kernel_stats.csv

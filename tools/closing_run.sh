#!/usr/bin/env bash
# Closing GPU call of a round: the full GPU test suite, smoke(), the default
# bench line (as the driver runs it), then bench + rocprof for small
# payload_cksum packets in 2048-B slots after the planner change.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/final2_pytest.log 2>&1 || { tail -40 gpurun_out/final2_pytest.log; exit 1; }
tail -1 gpurun_out/final2_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > gpurun_out/final2_smoke.log 2>&1 || { tail -20 gpurun_out/final2_smoke.log; exit 1; }
tail -1 gpurun_out/final2_smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final2_bench.json \
    2> gpurun_out/final2_bench.err || { tail -20 gpurun_out/final2_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/final2_bench.json').read().strip().splitlines()[-1]); r=d['roofline']
print('value', d['value'], 'frac', r['frac'], 'frac_rotating', r.get('frac_rotating'), 'c5', d.get('c5',{}).get('frac'))
print('c3', {k: v.get('frac') for k, v in d.get('c3', {}).get('sizes', {}).items()})
print('c4', d.get('c4', {}).get('frac') if isinstance(d.get('c4'), dict) else d.get('c4'))
"
CFGS="${CFGS:-s14pl_64 s14pl_128 s14pl_256 s14_64 s14_128}" TAG=${TAG:-r04c} bash tools/round_measure.sh \
    > gpurun_out/round_r04c.log 2>&1

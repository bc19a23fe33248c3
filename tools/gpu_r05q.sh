#!/usr/bin/env bash
# Round 5, call q: after the server-queue / library-lock changes -- the whole
# GPU suite, smoke(), the server's cost to a concurrent C2 batch again, and
# the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05q
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > $OUT/smoke.log 2>&1
rc=$?; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/serve_interference.py --rounds 5 > $OUT/interference.log 2>&1 \
    || { tail -20 $OUT/interference.log; exit 1; }
tail -5 $OUT/interference.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/bench.json'))
r = d['roofline']; print('C2', r['frac'], r['frac_job'], r.get('frac_rotating'), 'C5', d['c5']['frac_kernel'])
print('C3', {k: v['frac'] for k, v in d['c3']['sizes'].items()}, 'C4', d['c4']['frac'])
print('rings', {k: v['frac'] for k, v in d['rings'].items() if isinstance(v, dict)})"

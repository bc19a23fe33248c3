#!/usr/bin/env bash
# Round 5, call v: the shader clock beside every secondary bench leg
# (wc_sclk_probe) -- the bench test, then the default line twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05v
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_bench.py -k "one_gpu_line" tests/test_abi.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for k in 1 2; do
  timeout -k 10 400 python bench.py > $OUT/bench$k.json 2> $OUT/bench$k.err || { tail -20 $OUT/bench$k.err; exit 1; }
  python3 -c "
import json; d = json.load(open('$OUT/bench$k.json'))
r = d['roofline']; print('run $k C2', r['frac'], r['frac_job'], 'rot', r['rotating']['frac'], r['rotating']['sclk_MHz'], 'C5', d['c5']['frac_kernel'])
print('  C3', {k: (v['frac'], v['sclk_MHz']) for k, v in d['c3']['sizes'].items()}, 'C4', d['c4']['frac'], d['c4']['sclk_MHz'])
print('  rings', {k: (v['kernel_ms_avg_max_rank'], v['frac'], v['sclk_MHz']) for k, v in d['rings'].items() if isinstance(v, dict)})"
done

#!/usr/bin/env bash
# A/B of two library builds through bench.py (configs tune.py lacks, e.g. the
# RX verdict rings): WC_LIB=tools/libwccksum_prev.so (prev) vs the in-tree
# build (new), alternating, kernel time and roofline fraction per run.
#   ARGS_LIST="--config zrx;--config rx"  REPS=2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
IFS=';' read -ra LIST <<< "${ARGS_LIST:---config zrx}"
for a in "${LIST[@]}"; do
    echo "== $a"
    for rep in $(seq "${REPS:-2}"); do
        for which in prev new; do
            if [ $which = prev ]; then lib="WC_LIB=tools/libwccksum_prev.so"; else lib=""; fi
            env $lib timeout -k 10 200 python bench.py $a --steps 100 --warmup 20 --no-c5 \
                --no-cpu-baseline > gpurun_out/ab_bench.json 2> gpurun_out/ab_bench.err ||
                { tail gpurun_out/ab_bench.err; exit 1; }
            python -c "import json,sys; d=json.loads(open('gpurun_out/ab_bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$which', 'kernel %.2f us' % (1000*r['kernel_ms_avg']), 'frac %.4f' % r['frac'], 'parity', d.get('parity'))"
        done
    done
done

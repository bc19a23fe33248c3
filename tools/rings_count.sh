#!/usr/bin/env bash
# How often does a bench process land in the mixed rings' slow state?
# bench.py without the C5, e2e and CPU legs (the ring legs ride on the extra ones), REPS processes per
# library in LIBS, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-rings_count}
mkdir -p "$OUT"
for rep in $(seq 1 "${REPS:-4}"); do
    for lib in ${LIBS}; do
        WC_LIB="$lib" timeout -k 10 200 python bench.py ${BENCH_FLAGS:---no-c5 --no-e2e --no-cpu-baseline} \
            > "$OUT/r$rep.json" 2> "$OUT/r$rep.err" || exit 1
        python - "$OUT/r$rep.json" "$(basename "$lib")" "$rep" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["rings"]
print(f"rep{sys.argv[3]} {sys.argv[2]:18s} C2 {d['roofline']['frac']:.4f}", " ".join(
    f"{k} {v['frac']:.3f} ({v['kernel_ms_avg_max_rank'] * 1e3:.1f} us, {v['sclk_MHz']} MHz)"
    for k, v in r.items() if isinstance(v, dict)), flush=True)
PY
    done
done

#!/usr/bin/env bash
# Round 5, call h: the driver's default bench line, timed, with the RX ADAPT
# decisions traced; then bench lines + rocprofv3 kernel stats / FETCH_SIZE /
# WRITE_SIZE for C2, C5, the RX rings and C4 (tools/round_measure.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05h
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
t0=$(date +%s)
WC_RX_TRACE=1 timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json \
    2> $OUT/bench.err
rc=$?; echo "bench rc=$rc in $(( $(date +%s) - t0 )) s"; [ $rc -eq 0 ] || { grep -v "wccksum rx gen" $OUT/bench.err | tail; exit $rc; }
grep -c "wccksum rx gen" $OUT/bench.err
grep "wccksum rx gen" $OUT/bench.err | awk '{print $5}' | uniq -c | tail -12
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r05h/bench.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "frac", r["frac"], "frac_job", r["frac_job"], "rot", r.get("frac_rotating"))
print("c5", d["c5"]["frac_kernel"], d["c5"]["kernel_ms_avg_max_rank"])
print("c3", {k: v["frac"] for k, v in d["c3"]["sizes"].items()}, "c4", d["c4"]["frac"])
print("rings", {k: (v["frac"], v["kernel_ms_avg_max_rank"], v["steps"]) for k, v in d["rings"].items() if k != "workload"})
PY
CFGS="${CFGS:-c2 c5 zrx zrxa3 rx c4}" TAG=r05 bash tools/round_measure.sh > $OUT/round.log 2>&1
rc=$?; grep -E "^==|rc=" $OUT/round.log | tail -30; exit $rc

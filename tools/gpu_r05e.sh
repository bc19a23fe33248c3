#!/usr/bin/env bash
# Round 5, call e: parity of the split launches (the C5 full-size test
# included), the driver's default bench line (headline + c3/c4/c5/rings),
# then the server-interference and host-latency runs (call c).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05e
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "split or c5 or bench" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; [ $rc -eq 0 ] || { tail -20 $OUT/bench.err; exit $rc; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r05e/bench.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "frac", r["frac"], "frac_job", r["frac_job"], "rot", r.get("frac_rotating"))
print("c5", d["c5"]["frac_kernel"], d["c5"]["kernel_ms_avg_max_rank"], d["c5"]["parity"])
print("c3", {k: v["frac"] for k, v in d["c3"]["sizes"].items()}, "c4", d["c4"]["frac"])
print("rings", {k: (v["frac"], v["kernel_ms_avg_max_rank"]) for k, v in d["rings"].items() if k != "workload"})
print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["value_1core"], "parity", d["parity"])
PY
R05C_OUT=r05e bash tools/gpu_r05c.sh

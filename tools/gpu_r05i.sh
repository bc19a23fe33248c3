#!/usr/bin/env bash
# Round 5, call i: the bench tests and the default line after the C5 leg's
# longer warm-up / timed window; 9000-B packets (9.4 GB, three 3-GiB pieces
# by default) against other split sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05i
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; [ $rc -eq 0 ] || { tail $OUT/bench.err; exit $rc; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r05i/bench.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "frac", r["frac"], "frac_job", r["frac_job"], "rot", r.get("frac_rotating"))
print("c5", d["c5"]["frac_kernel"], d["c5"]["kernel_ms_avg_max_rank"], d["c5"]["steps"], d["c5"]["warmup_steps"])
print("c3", {k: v["frac"] for k, v in d["c3"]["sizes"].items()}, "c4", d["c4"]["frac"])
print("rings", {k: v["frac"] for k, v in d["rings"].items() if k != "workload"})
PY
timeout -k 10 300 python tools/tune.py --config c3 --len 9000 --rounds 4 --iters 10 \
    --variants "default;WC_SPLIT_BYTES=0;WC_SPLIT_BYTES=1610612736;WC_SPLIT_BYTES=6442450944" \
    > $OUT/c3_9000_split.log 2>&1 || exit 1
grep -v "amdgpu.ids" $OUT/c3_9000_split.log | grep -v "^ *round"

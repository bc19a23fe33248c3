#!/usr/bin/env bash
# Does the bench line's e2e leg read slower after the device-resident legs?
# The e2e leg alone (bench.py with every other leg off), twice, then
# tools/e2e.py (the same leg in a fresh process) on the product library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-e2e_order}
mkdir -p "$OUT"
for i in 1 2; do
    timeout -k 10 200 python bench.py --no-c5 --no-extra --no-rings --no-cpu-baseline \
        > "$OUT/e2e_only_$i.json" 2> "$OUT/e2e_only_$i.err" || exit 1
    python - "$OUT/e2e_only_$i.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["e2e"]
print("e2e leg alone: H2D", e["h2d_ceiling_GBps"]["pinned"],
      [(k, v["registered"]["GBps"], v["pageable"]["GBps"]) for k, v in e["calls"].items()])
PY
done
WC_TUNING=0 timeout -k 10 200 python tools/e2e.py --reps 5 2>&1 | grep "^{" | tee "$OUT/e2e_tool.jsonl"

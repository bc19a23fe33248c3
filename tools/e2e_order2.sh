#!/usr/bin/env bash
# Which device-resident leg slows the bench line's e2e leg?  bench.py with
# one group of legs at a time before the e2e leg (cpu baseline off).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export WC_NO_BUILD=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-e2e_order2}
mkdir -p "$OUT"
run() {  # $1 = name, rest = bench flags
    local name=$1; shift
    timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || exit 1
    python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["e2e"]
print(sys.argv[2], "H2D", e["h2d_ceiling_GBps"]["pinned"],
      [(k, v["registered"]["GBps"], v["pageable"]["GBps"]) for k, v in e["calls"].items()])
PY
}
run only_c5 --no-extra --no-rings
run only_extra --no-c5 --no-rings
run only_rings --no-c5 --no-extra
run all

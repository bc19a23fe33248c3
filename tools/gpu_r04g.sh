#!/usr/bin/env bash
# Round-4 pass g: C3 small sizes from HBM -- fewer bytes per wave (more,
# shorter waves) under rocprofv3, rotating 1 GiB of buffers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$PWD
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp WC_NO_BUILD=1
run_prof() {  # $1 = name, rest = tune.py args
  local name=$1; shift
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$REPO/$O/prof_$name" -o run --output-format csv -- python3 "$REPO/tools/tune.py" "$@") > $O/prof_$name.log 2>&1 || { tail $O/prof_$name.log; exit 1; }
  rm -f $O/prof_$name/run_kernel_trace.csv
  python3 - "$O/prof_$name/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "synth" in r["Name"] or "rocclr" in r["Name"]:
        continue
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    print(f'   {n:<60} calls {r["Calls"]:>7} avg {float(r["AverageNs"])/1000:8.2f} us')
PY
}
G="--rotate-bytes 1073741824 --rounds 3 --iters 300 --warm-ms 30"
echo "== 64"; run_prof c3_64 --config c3 --len 64 $G --variants "default;WC_SHAPE=4,1,2;WC_LEAN_MAX=0 WC_SHAPE=4,1,1;WC_LEAN_MAX=0 WC_SHAPE=4,1,2;WC_LEAN_MAX=0 WC_SHAPE=8,1,2"
echo "== 128"; run_prof c3_128 --config c3 --len 128 $G --variants "default;WC_SHAPE=8,1,2;WC_LEAN_MAX=0 WC_SHAPE=16,1,2;WC_LEAN_MAX=0 WC_SHAPE=8,1,2;WC_SHAPE=16,1,4"
echo "== 256"; run_prof c3_256 --config c3 --len 256 $G --variants "default;WC_SHAPE=16,1,4;WC_SHAPE=16,2,2;WC_LEAN_MAX=0 WC_SHAPE=16,1,2;WC_SHAPE=8,2,4"
echo "== 64 B plain read ceiling from HBM (tune.py --ceiling, HIP events incl. launch gaps)"
timeout -k 10 300 python3 tools/tune.py --config c3 --len 64 --rotate-bytes 1073741824 --rounds 2 --iters 200 --warm-ms 20 --ceiling > $O/ceiling_64.log 2>&1 || { tail $O/ceiling_64.log; exit 1; }
grep -v amdgpu $O/ceiling_64.log | grep -v TILEREAD

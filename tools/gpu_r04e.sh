#!/usr/bin/env bash
# Round-4 pass e: server latency after overlapping its record loads; C3
# small sizes from HBM (rotating buffers): kernel shapes under rocprofv3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$PWD
O=gpurun_out/r04e
mkdir -p $O
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "host_ or rx_verdict_host or c_rx or c_host or netmap_ring" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for W in 64 128; do
  WC_SERVE_WAVES=$W timeout -k 10 200 build/host_latency 16 0.2 > $O/host_latency_w$W.log 2>&1 || { tail $O/host_latency_w$W.log; exit 1; }
  echo "== waves $W"; cut -c1-130 $O/host_latency_w$W.log | head -4; sed -n 7,10p $O/host_latency_w$W.log | cut -c1-130
done
run_prof() {  # $1 = name, rest = tune.py args
  local name=$1; shift
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$REPO/$O/prof_$name" -o run --output-format csv -- python3 "$REPO/tools/tune.py" "$@") > $O/prof_$name.log 2>&1 || { tail $O/prof_$name.log; exit 1; }
  rm -f $O/prof_$name/run_kernel_trace.csv
  python3 - "$O/prof_$name/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "synth" in r["Name"] or "rocclr" in r["Name"]:
        continue
    print(f'   {r["Name"].split("(")[0][-60:]:<60} calls {r["Calls"]:>7} avg {float(r["AverageNs"])/1000:8.2f} us')
PY
}
for L in 64 128 256; do
  echo "== C3 $L B, rotating 1 GiB"
  run_prof c3_$L --config c3 --len $L --rotate-bytes 1073741824 --rounds 3 --iters 300 --warm-ms 30 --variants "default;WC_NT=0;WC_LEAN_MAX=0;WC_LEAN_MAX=0 WC_SHAPE=4,1,8;WC_LEAN_MAX=0 WC_SHAPE=4,1,16;WC_LEAN_MAX=0 WC_SHAPE=8,1,8;WC_LEAN_MAX=0 WC_SHAPE=16,1,8"
done

#!/bin/bash
# SURVEY config 1 (sockping -> echo over loopback) with and without the GPU
# verify pass on the socket RX path: builds tests/c/sock_verify.c and runs it
# for 1 payload per round trip (ping.c's shape) and for w_rx-sized batches.
#   tools/sock_bench.sh [loops]      -> one JSON line per configuration, and
#   sockping-format TSVs (bin/ping.c:215, 301-302) in $TSV_DIR (default
#   gpurun_out/): ping_b<batch>_s<len>.{off,on}.tsv
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
LOOPS="${1:-20000}"
EXE="${TMPDIR:-/tmp}/sock_verify.$$"
gcc -O2 -std=gnu11 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -I"$ROOT/include" \
    -I"$ROOT/oracle" "$ROOT/tests/c/sock_verify.c" "$ROOT/oracle/wc_oracle.c" -o "$EXE" \
    -L"$ROOT/warpcore_amd" -lwccksum -L/opt/rocm/lib -lamdhip64 -lpthread \
    -Wl,-rpath,"$ROOT/warpcore_amd"
TSV_DIR="${TSV_DIR:-$ROOT/gpurun_out}"
mkdir -p "$TSV_DIR"
for cfg in "1 1472" "64 1472" "1 64" "64 64"; do
    set -- $cfg
    timeout -k 10 300 "$EXE" -b "$1" -s "$2" -l "$LOOPS" -t "$TSV_DIR/ping_b$1_s$2"
done
rm -f "$EXE"

#!/usr/bin/env bash
# Round 4: does a capped grid (several tiles per wave) lose C4 time because
# the next tile's loads wait on the previous tile's result store?  Capped
# grids with and without the result store (tuning build: WC_VARIANT bits
# 20-23 = k -> k x 1024 blocks, bit 24 = no result store).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
NS=$((1 << 24))
V="default;WC_VARIANT=$NS"
for k in 2 4 8 12; do
  V="$V;WC_VARIANT=$((k << 20));WC_VARIANT=$((k << 20 | NS))"
done
timeout -k 10 400 python3 tools/tune.py --rounds 3 --iters 10 --config c4 \
  --variants "$V" > gpurun_out/r04h_c4_cap.log 2>&1

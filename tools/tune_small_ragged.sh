#!/bin/bash
# Small ragged (Zipf) batches: flat kernel vs the ragged group kernel shapes.
set -euo pipefail
cd "$(dirname "$0")/.."
G="WC_FLAT_MIN=1000000000"
for n in ${SIZES:-64 1024 8192 32768 131072 524288 2097152}; do
    echo "== c4 zipf, $n packets"
    python tools/tune.py --config c4 --packets "$n" --rounds 5 --iters 50 \
        --variants "WC_FLAT_MIN=0;$G;$G WC_RAGGED_SHAPE=32,2,1;$G WC_RAGGED_SHAPE=16,2,2;$G WC_RAGGED_SHAPE=64,4,1"
done

#!/usr/bin/env bash
# A/B/C of several library builds on the GPU box, alternating fresh processes:
#   LIBS="tools/a.so tools/b.so warpcore_amd/libwccksum.so"
#   CASES="--config zrx;--config zrx --rx-arp 3"   (tune.py arguments, ';'-separated)
#   REPS=3  OUT=gpurun_out/ab_libs.log
# Each line: rep, case number, library, then tune.py's median line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1 WC_TUNING=0
OUT=${OUT:-gpurun_out/ab_libs.log}
IFS=';' read -ra cases <<< "${CASES:---config zrx}"
for rep in $(seq 1 "${REPS:-3}"); do
    c=0
    for a in "${cases[@]}"; do
        c=$((c + 1))
        for lib in ${LIBS}; do
            line=$(WC_LIB="$lib" timeout -k 10 120 python tools/tune.py $a --rounds 3 --iters 20 2>&1 \
                   | grep -v amdgpu.ids | tail -1) || { echo "FAILED: $lib $a"; exit 1; }
            echo "rep$rep case$c $(basename "$lib") $line" | tee -a "$OUT"
        done
    done
done

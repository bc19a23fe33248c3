#!/usr/bin/env bash
# A/B of two library builds (separate processes, alternating):
#   WC_LIB=tools/libwccksum_prev.so (A) vs the in-tree build (B).
#   CASES="c4:payload rslot:payload"  ROUNDS=4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
T="timeout -k 10 120 python tools/tune.py --rounds ${ROUNDS:-4} --iters 20"
for c in ${CASES:-c4:payload}; do
    cfg=${c%%:*}; kind=${c##*:}; hdr=""
    case $kind in
        payload+h) kind=payload; hdr="--headers" ;;
        fused) kind=payload; hdr="--headers --fused" ;;
    esac
    case $cfg in
        c2) a="--config c2" ;;
        c4) a="--config c4" ;;
        zslots) a="--config zslots" ;;
        slot) a="--config c3 --len 1500 --stride 2048 --offset 14" ;;
        rslot) a="--config c3 --len 1500 --stride 2048 --offset 14 --ragged" ;;
        rc2) a="--config c2 --ragged" ;;
        c3-*) a="--config c3 --len ${cfg#c3-}" ;;
        s14-*) a="--config c3 --len ${cfg#s14-} --stride 2048 --offset 14" ;;
    esac
    echo "== $c"
    for rep in 1 2; do
        echo -n "prev "; WC_LIB=tools/libwccksum_prev.so $T $a --kind $kind $hdr 2>&1 | grep -v amdgpu.ids || exit 1
        echo -n "new  "; $T $a --kind $kind $hdr 2>&1 | grep -v amdgpu.ids || exit 1
    done
done

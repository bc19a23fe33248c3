#!/usr/bin/env bash
# A/B timing of kernel variants on the GPU box (parity first with VP set).
#   VP="WC_VARIANT=4"  env for the parity pass (optional)
#   CASES="c2:ip c2:payload c3-64:ip slot:ip slot:payload c4:ip c4:payload"
#   VARS="default;WC_VARIANT=4"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
if [ -n "${VP:-}" ]; then
    env $VP timeout -k 10 300 python -m pytest tests -m gpu -x -q --timeout 120 \
        --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
    tail -1 gpurun_out/ab_pytest.log
fi
T="timeout -k 10 200 python tools/tune.py --rounds ${ROUNDS:-6} --iters 20"
for c in ${CASES:-c2:ip c2:payload}; do
    cfg=${c%%:*}; kind=${c##*:}; hdr=""
    case $kind in
        payload+h) kind=payload; hdr="--headers" ;;
        fused) kind=payload; hdr="--headers --fused" ;;
    esac
    case $cfg in
        c2) a="--config c2" ;;
        c4) a="--config c4" ;;
        c4r) a="--config c4r" ;;
        zslots) a="--config zslots" ;;
        slot) a="--config c3 --len 1500 --stride 2048 --offset 14" ;;
        rslot) a="--config c3 --len 1500 --stride 2048 --offset 14 --ragged" ;;
        rc2) a="--config c2 --ragged" ;;
        c3-*) a="--config c3 --len ${cfg#c3-}" ;;
        s14-*) a="--config c3 --len ${cfg#s14-} --stride 2048 --offset 14" ;;
    esac
    echo "== $c"
    log=gpurun_out/ab_${cfg}_${kind}${hdr:+_h}.log
    $T $a --kind $kind $hdr --variants "$VARS" > $log 2>&1 || { tail $log; exit 1; }
    grep -v "^\s*round\|amdgpu.ids" $log
done

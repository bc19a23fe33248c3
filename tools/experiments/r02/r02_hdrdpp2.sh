#!/usr/bin/env bash
# payload group kernel, 4- and 8-lane groups: DPP header broadcast (default) vs ds_bpermute (WC_VARIANT bit 19),
# and against the seg kernel the planner picks for packed batches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/hd2_pytest.log 2>&1 || { tail -40 gpurun_out/hd2_pytest.log; exit 1; }
tail -1 gpurun_out/hd2_pytest.log
T="timeout -k 10 120 python tools/tune.py --rounds 4 --iters 20 --warm-ms 20 --kind payload --headers"
V="default;WC_STRIDED_SEG=0 WC_VARIANT=524288;WC_STRIDED_SEG=0"
for L in 64 100 128 192 256; do echo "### payload $L packed (seg / group bpermute / group DPP)"; $T --config c3 --len $L --variants "$V" 2>&1 | grep -v amdgpu.ids || exit 1; done
for L in 64 256; do echo "### payload $L in 2048-B slots +14 (group bpermute / group DPP)"; $T --config c3 --len $L --stride 2048 --offset 14 --variants "WC_VARIANT=524288;default" 2>&1 | grep -v amdgpu.ids || exit 1; done

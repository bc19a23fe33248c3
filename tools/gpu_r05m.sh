#!/usr/bin/env bash
# Round 5, call m: (1) several engines on threads calling the library at once
# (tests/c/thread_engines.c); (2) the mixed-size RX ring against the plain
# ragged payload_cksum of the same 2^21 Zipf lengths, in slots and packed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05m
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
    tests/test_gpu_rx.py -k "thread_engines" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
gcc -O2 -std=gnu11 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -Ioracle \
    tests/c/thread_engines.c oracle/wc_oracle.c -o /tmp/thread_engines -Lwarpcore_amd -lwccksum \
    -L/opt/rocm/lib -lamdhip64 -lpthread -Wl,-rpath,$PWD/warpcore_amd || exit 1
timeout -k 10 60 /tmp/thread_engines 8 8 3 > $OUT/threads.log 2>&1 || { cat $OUT/threads.log; exit 1; }
cat $OUT/threads.log
T="timeout -k 10 300 python tools/tune.py --rounds 4 --iters 20"
{ echo "== zrx slots"; $T --config zrx; } >> $OUT/rxframe.log 2>&1 || exit 1
{ echo "== zrx packed"; $T --config zrx --rx-packed; } >> $OUT/rxframe.log 2>&1 || exit 1
{ echo "== zslots payload (the same ip lengths at +14 of 2048-B slots)"; $T --config zslots --kind payload --headers; } >> $OUT/rxframe.log 2>&1 || exit 1
{ echo "== c4 payload 2^21 packed"; $T --config c4 --packets 2097152 --kind payload --headers; } >> $OUT/rxframe.log 2>&1 || exit 1
{ echo "== c4 ip 2^21 packed"; $T --config c4 --packets 2097152; } >> $OUT/rxframe.log 2>&1 || exit 1
grep -E "^==|default" $OUT/rxframe.log

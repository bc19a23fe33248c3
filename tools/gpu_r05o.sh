#!/usr/bin/env bash
# Round 5, call o: the first-come-first-served library lock and the lock-free
# device-call entry -- thread_engines (no starvation), the host-path GPU
# tests, and the host latency table (the lock's cost on a single engine).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05o
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
    tests/test_gpu_rx.py tests/test_gpu_parity.py -k "thread_engines or host or server or tx_queue" \
    > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
gcc -O2 -g -rdynamic -std=gnu11 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -Ioracle \
    tests/c/thread_engines.c oracle/wc_oracle.c -o /tmp/thread_engines -Lwarpcore_amd -lwccksum \
    -L/opt/rocm/lib -lamdhip64 -lpthread -Wl,-rpath,$PWD/warpcore_amd || exit 1
timeout -k 10 60 /tmp/thread_engines 8 8 3 > $OUT/threads.log 2>&1 || { cat $OUT/threads.log; exit 1; }
cat $OUT/threads.log
python3 -c "import sys; sys.path.insert(0, 'tests'); from cprog import build; build('host_latency', '$OUT')" \
    || exit 1
timeout -k 10 400 $OUT/host_latency 16 0.4 > $OUT/host_latency.log 2>&1
rc=$?; cat $OUT/host_latency.log | tail -40; exit $rc

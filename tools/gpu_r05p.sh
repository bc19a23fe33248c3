#!/usr/bin/env bash
# Round 5, call p: the server grid on a highest-priority stream (no shared
# hardware queue) -- the new test, its A/B against the old normal-priority
# stream (expected to stall), thread_engines, the host-path tests and the
# host latency table.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05p
mkdir -p $OUT
export TMPDIR=/tmp WC_NO_BUILD=1
PT="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 200 $PT tests/test_gpu_parity.py -k "grid_holds_up" > $OUT/prio.log 2>&1 \
    || { tail -30 $OUT/prio.log; exit 1; }
tail -2 $OUT/prio.log
WC_SERVE_PRIO=0 timeout -k 10 200 $PT tests/test_gpu_parity.py -k "grid_holds_up" > $OUT/prio0.log 2>&1
rc=$?
echo "WC_SERVE_PRIO=0 (old stream): pytest rc=$rc"; grep -E "AssertionError|assert dt|^E " $OUT/prio0.log | head -5
case $rc in 0|1) ;; *) exit 1 ;; esac
gcc -O2 -g -rdynamic -std=gnu11 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -Ioracle \
    tests/c/thread_engines.c oracle/wc_oracle.c -o /tmp/thread_engines -Lwarpcore_amd -lwccksum \
    -L/opt/rocm/lib -lamdhip64 -lpthread -Wl,-rpath,$PWD/warpcore_amd || exit 1
timeout -k 10 60 /tmp/thread_engines 8 8 3 > $OUT/threads.log 2>&1 || { cat $OUT/threads.log; exit 1; }
cat $OUT/threads.log
timeout -k 10 400 $PT tests/test_gpu_rx.py tests/test_gpu_parity.py \
    -k "thread_engines or host or server or tx_queue" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
python3 -c "import sys; sys.path.insert(0, 'tests'); from cprog import build; build('host_latency', '$OUT')" \
    || exit 1
timeout -k 10 400 $OUT/host_latency 16 0.4 > $OUT/host_latency.log 2>&1
rc=$?; tail -40 $OUT/host_latency.log; exit $rc

#!/usr/bin/env bash
# Round 5, call n: thread_engines with a crash backtrace (call m: SIGSEGV
# within ~1 s, no output).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05n
mkdir -p $OUT
gcc -O2 -g -rdynamic -std=gnu11 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -Ioracle \
    tests/c/thread_engines.c oracle/wc_oracle.c -o /tmp/thread_engines -Lwarpcore_amd -lwccksum \
    -L/opt/rocm/lib -lamdhip64 -lpthread -Wl,-rpath,$PWD/warpcore_amd || exit 1
timeout -k 10 60 /tmp/thread_engines 4 4 2 > $OUT/threads.log 2>&1
rc=$?
echo "rc=$rc" >> $OUT/threads.log
cat $OUT/threads.log
exit 0

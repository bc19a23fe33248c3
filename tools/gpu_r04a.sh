#!/usr/bin/env bash
# Round-4 first GPU pass: new GPU tests (bench legs, re-register, resident
# server, RX modes, C programs), the default bench line, C3 64 B rotating,
# the C latency tool, RX-mode and C4 store A/Bs, the counter list.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04a
export TMPDIR=/tmp WC_NO_BUILD=1
O=gpurun_out/r04a
timeout -k 10 700 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_parity.py tests/test_gpu_rx.py -x -v --timeout 300 --timeout-method thread -k "one_gpu_line or c3_rotating or two_ranks or host_ or zero_copy or rx_ or c_host_latency" > $O/t_bench.log 2>&1 || { tail -40 $O/t_bench.log; exit 1; }
tail -3 $O/t_bench.log
WC_SERVE_MAX=1024 timeout -k 10 120 build/rx_ring_loop 4 1024 > $O/rx_ring_srv.log 2>&1 || { cat $O/rx_ring_srv.log; exit 1; }
cat $O/rx_ring_srv.log
timeout -k 10 200 build/host_latency 16 0.3 > $O/host_latency.log 2>&1 || { tail $O/host_latency.log; exit 1; }
cat $O/host_latency.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
timeout -k 10 200 python bench.py --config c3 --len 64 --no-c5 --no-cpu-baseline > $O/c3_64.json 2>&1 || exit 1
V="default;WC_RX_ROWS=2;WC_RX_EARLY=1;WC_RX_ROWS=2 WC_RX_EARLY=1"
for a in "--config zrx" "--config rx" "--config zrx --rx-arp 3"; do
  echo "== tune $a" >> $O/tune_rx.log
  timeout -k 10 200 python tools/tune.py $a --rounds 5 --iters 20 --variants "$V" >> $O/tune_rx.log 2>&1 || exit 1
done
grep -v amdgpu $O/tune_rx.log
echo "== C4 store A/B (tuning build: bit 24 drops the result store)" >> $O/tune_store.log
timeout -k 10 200 python tools/tune.py --config c4 --rounds 5 --iters 10 --variants "default;WC_VARIANT=16777216" >> $O/tune_store.log 2>&1 || exit 1
grep -v amdgpu $O/tune_store.log
(cd /tmp && timeout -k 10 60 rocprofv3 -L) > $O/counters.txt 2>&1 || true
grep -c . $O/counters.txt

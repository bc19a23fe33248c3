set -u
mkdir -p gpurun_out/r04a
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_parity.py tests/test_gpu_rx.py -x -v --timeout 300 --timeout-method thread -k "one_gpu_line or c3_rotating or two_ranks or host_register or zero_copy or rx_ or c_host_latency" > gpurun_out/r04a/t_bench.log 2>&1 || { tail -30 gpurun_out/r04a/t_bench.log; exit 1; }
tail -3 gpurun_out/r04a/t_bench.log
timeout -k 10 300 python bench.py > gpurun_out/r04a/bench_default.json 2> gpurun_out/r04a/bench_default.err || { tail gpurun_out/r04a/bench_default.err; exit 1; }
timeout -k 10 200 python bench.py --config c3 --len 64 --no-c5 --no-cpu-baseline > gpurun_out/r04a/c3_64.json 2>&1 || exit 1
timeout -k 10 200 build/host_latency 16 0.3 > gpurun_out/r04a/host_latency.log 2>&1 || exit 1
V="default;WC_RX_ROWS=2;WC_RX_EARLY=1;WC_RX_ROWS=2 WC_RX_EARLY=1"
for a in "--config zrx" "--config rx" "--config zrx --rx-arp 3"; do
  echo "== tune $a" >> gpurun_out/r04a/tune_rx.log
  timeout -k 10 200 python tools/tune.py $a --rounds 5 --iters 20 --variants "$V" >> gpurun_out/r04a/tune_rx.log 2>&1 || exit 1
done
cat gpurun_out/r04a/tune_rx.log | grep -v amdgpu
echo "== C4 store A/B (tuning build: bit 24 drops the result store)" >> gpurun_out/r04a/tune_store.log
timeout -k 10 200 python tools/tune.py --config c4 --rounds 5 --iters 10 --variants "default;WC_VARIANT=16777216" >> gpurun_out/r04a/tune_store.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/r04a/tune_store.log
(cd /tmp && timeout -k 10 60 rocprofv3 -L) > gpurun_out/r04a/counters.txt 2>&1 || true
grep -c . gpurun_out/r04a/counters.txt

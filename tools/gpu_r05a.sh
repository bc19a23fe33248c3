set -u
mkdir -p gpurun_out/r05a
export TMPDIR=/tmp WC_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rx.py -x -v --timeout 120 --timeout-method thread -k "fused or server or host or rx or tx_queue" > gpurun_out/r05a/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r05a/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/c5_clock.py --rounds 3 > gpurun_out/r05a/c5clock.log 2>&1
rc=$?; tail -12 gpurun_out/r05a/c5clock.log; exit $rc

set -e
mkdir -p gpurun_out
T="timeout -k 10 300 python tools/tune.py --rounds 6 --iters 20"
$T --config c3 --len 64 --variants "default;WC_SHAPE=4,1,16;WC_SHAPE=8,1,4;WC_SHAPE=8,1,8;WC_SHAPE=4,1,8 WC_NT=0" > gpurun_out/c3_64.log 2>&1
$T --config c3 --len 256 --variants "default;WC_SHAPE=16,1,8;WC_SHAPE=16,2,4;WC_SHAPE=8,1,8" > gpurun_out/c3_256.log 2>&1
$T --config c3 --len 576 --variants "default;WC_SHAPE=16,6,2;WC_SHAPE=16,3,4 WC_NT=0" > gpurun_out/c3_576.log 2>&1
$T --config c3 --len 1472 --variants "default;WC_SHAPE=32,3,8;WC_SHAPE=32,3,4;WC_SHAPE=16,6,2" > gpurun_out/c3_1472.log 2>&1
$T --config c3 --len 9000 --variants "default;WC_SHAPE=64,9,1;WC_SHAPE=64,9,2;WC_SHAPE=64,4,1" > gpurun_out/c3_9000.log 2>&1

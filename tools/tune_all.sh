set -e
mkdir -p gpurun_out
T="timeout -k 10 300 python tools/tune.py --rounds 5 --iters 20"
$T --config c3 --len 64 --variants "WC_SHAPE=4,1,4;WC_SHAPE=4,1,8;WC_SHAPE=4,1,16;WC_SHAPE=8,1,4;WC_SHAPE=8,1,8" > gpurun_out/t64.log 2>&1
$T --config c3 --len 256 --variants "WC_SHAPE=16,1,4;WC_SHAPE=16,1,8;WC_SHAPE=8,2,4;WC_SHAPE=16,2,2;WC_SHAPE=16,2,4" > gpurun_out/t256.log 2>&1
$T --config c3 --len 576 --variants "WC_SHAPE=16,3,2;WC_SHAPE=16,3,4;WC_SHAPE=16,4,2;WC_SHAPE=32,2,1;WC_SHAPE=16,6,2" > gpurun_out/t576.log 2>&1
$T --config c2 --variants "WC_SHAPE=32,3,4;WC_SHAPE=32,3,8;WC_SHAPE=16,6,2;WC_SHAPE=16,6,4;WC_SHAPE=32,3,2" > gpurun_out/t1472.log 2>&1
$T --config c3 --len 9000 --variants "WC_SHAPE=64,9,1;WC_SHAPE=64,9,2;WC_SHAPE=32,18,1;WC_SHAPE=64,8,1;WC_SHAPE=64,4,1" > gpurun_out/t9000.log 2>&1
$T --config c4 --variants "WC_SHAPE=16,2,2;WC_SHAPE=16,2,4;WC_SHAPE=16,4,2;WC_SHAPE=8,2,4;WC_SHAPE=16,1,8;WC_SHAPE=32,3,1;WC_SHAPE=16,3,4" > gpurun_out/tzipf.log 2>&1

#!/bin/bash
# Round-2 probes: lane-pattern read rates and the current below-roofline cases.
set -e
export WC_NO_BUILD=1
mkdir -p gpurun_out
timeout -k 10 120 python tools/pattern_probe.py > gpurun_out/pattern.log 2>&1
T="timeout -k 10 150 python tools/tune.py --rounds 5 --iters 20"
$T --config zslots --variants "default;WC_SEG=0" > gpurun_out/zslots_ip.log 2>&1
$T --config zslots --kind payload --headers --variants "default;WC_SEG=0" > gpurun_out/zslots_pl.log 2>&1
$T --config c3 --len 64 > gpurun_out/c3_64.log 2>&1
$T --config c3 --len 256 --offset 14 > gpurun_out/c3_256o14.log 2>&1
$T --config c3 --len 100 > gpurun_out/c3_100.log 2>&1
$T --config c3 --len 9000 > gpurun_out/c3_9000.log 2>&1

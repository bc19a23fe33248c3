#!/bin/bash
set -e
export WC_NO_BUILD=1
mkdir -p gpurun_out
T="timeout -k 10 150 python tools/tune.py --rounds 5 --iters 20"
V="WC_SEG=0;WC_SEG=0 WC_FLAT_PK=2;WC_SEG=0 WC_FLAT_PK=2 WC_FLAT_UN=1;WC_SEG=0 WC_FLAT_PK=2 WC_FLAT_UN=4;default"
$T --config zslots --variants "$V" > gpurun_out/pk_zslots_ip.log 2>&1
$T --config zslots --kind payload --headers --variants "$V" > gpurun_out/pk_zslots_pl.log 2>&1
$T --config c4 --variants "$V" > gpurun_out/pk_c4.log 2>&1

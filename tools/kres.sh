#!/usr/bin/env bash
# VGPR count and occupancy of every kernel in wc_cksum_kernels.hip (gfx950).
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -c --offload-device-only \
    -Rpass-analysis=kernel-resource-usage -Iinclude -Iwarpcore_amd/csrc \
    warpcore_amd/csrc/wc_cksum_kernels.hip -o /tmp/wc_kres.o 2>&1 |
    sed 's/.*remark: //; s/ \[-Rpass.*//' |
    awk '/Function Name/{name=$3} /^ *VGPRs:/{v=$2} /ScratchSize/{sc=$NF} /Occupancy/{print name, "vgpr", v, "scratch", sc, "occ", $NF}' |
    c++filt | sed 's/void wc::k_cksum_//; s/(.*)//' | grep -E "${1:-.}"

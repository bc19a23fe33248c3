#!/usr/bin/env bash
# VGPR count, scratch and occupancy of every kernel in the wc_k_*.hip
# translation units (gfx950).  Optional argument: a regex over the names.
cd "$(dirname "$0")/.."
for f in warpcore_amd/csrc/wc_k_*.hip; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -c --offload-device-only \
        -Rpass-analysis=kernel-resource-usage -Iinclude -Iwarpcore_amd/csrc \
        "$f" -o /tmp/wc_kres.o 2>&1
done |
    sed 's/.*remark: //; s/ \[-Rpass.*//' |
    awk '/Function Name/{name=$3} /^ *VGPRs:/{v=$2} /ScratchSize/{sc=$NF} /Occupancy/{print name, "vgpr", v, "scratch", sc, "occ", $NF}' |
    c++filt | sed 's/void wc::\((anonymous namespace)::\)\?k_cksum_//; s/(.*)//' | grep -E "${1:-.}"

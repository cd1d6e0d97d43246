#!/bin/bash
# Build timing-only variants of libtwotower_hip.so (results wrong) for the ring filter A/B.
set -e
cd "$(dirname "$0")/../two-tower-model-v2_amd/csrc"
mkdir -p ../lib/variants ../build/variants
for v in "base:" "nodma:-DTT_EXP_NODMA=1" "nosel:-DTT_EXP_NOSEL=1" "nobar:-DTT_EXP_NOBAR=1" "nodma_nosel:-DTT_EXP_NODMA=1 -DTT_EXP_NOSEL=1"; do
  name=${v%%:*}; defs=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $defs -x hip -c tt_filter.hip -o ../build/variants/tt_filter_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC ../build/tt_common.cpp.o ../build/tt_norm.hip.o ../build/tt_scan.hip.o ../build/tt_buyer.hip.o ../build/variants/tt_filter_$name.o -o ../lib/variants/lib_$name.so
done
ls -la ../lib/variants

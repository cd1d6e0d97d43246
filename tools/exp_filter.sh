#!/bin/bash
# Build timing-only variants of libtwotower_hip.so (results wrong) for the ring filter A/B.
set -e
cd "$(dirname "$0")/../two-tower-model-v2_amd/csrc"
mkdir -p ../lib/variants ../build/variants
VARIANTS=${VARIANTS:-"base: nosel:-DTT_EXP_NOSEL=1 nowrite:-DTT_EXP_NOWRITE=1 maxonly:-DTT_EXP_MAXONLY=1"}
# (skipping the DMA or the per-tile barrier left garbage candidate rows: memory faults in the
# re-rank, so those switches were removed)
FILE=${FILE:-tt_filter}  # the source the variants differ in (tt_filter or tt_encoder)
rm -f ../lib/variants/lib_*.so
for v in $VARIANTS; do
  name=${v%%:*}; defs=${v#*:}; defs=${defs//,/ }
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DTT_TIMING_BUILD $defs -x hip -c $FILE.hip -o ../build/variants/${FILE}_$name.o
  others=$(ls ../build/*.o | grep -v $FILE)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $others ../build/variants/${FILE}_$name.o -o ../lib/variants/lib_$name.so
done
ls -la ../lib/variants

#!/bin/bash
# Build variants that differ in compile flags of BOTH tt_filter.hip and tt_encoder.hip.
#   VARIANTS="name:-DA=1,-DB=2 ..." bash tools/exp_build2.sh
set -e
cd "$(dirname "$0")/../two-tower-model-v2_amd/csrc"
mkdir -p ../lib/variants ../build/variants
rm -f ../lib/variants/lib_*.so
for v in $VARIANTS; do
  name=${v%%:*}; defs=${v#*:}; defs=${defs//,/ }
  for f in ${EXP_FILES:-tt_filter tt_encoder tt_scan}; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DTT_TIMING_BUILD $defs -x hip -c $f.hip -o ../build/variants/${f}_$name.o 2>/dev/null &
  done
  wait
  objs=""
  others=$(ls ../build/*.o)
  for f in ${EXP_FILES:-tt_filter tt_encoder tt_scan}; do
    others=$(echo "$others" | grep -v "/$f\.")
    objs="$objs ../build/variants/${f}_$name.o"
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $others $objs -o ../lib/variants/lib_$name.so
done
ls ../lib/variants

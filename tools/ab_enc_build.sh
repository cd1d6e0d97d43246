#!/bin/bash
# A/B builds of tt_encoder.hip: lib_o from git HEAD (or $OLD_REV), lib_n from the working tree,
# both timing builds (TT_TIMING_BUILD) linked with the in-tree objects of the other files.
set -e
cd "$(dirname "$0")/../two-tower-model-v2_amd/csrc"
mkdir -p ../lib/variants ../build/variants /tmp/ab_old
git show ${OLD_REV:-HEAD}:two-tower-model-v2_amd/csrc/tt_encoder.hip > /tmp/ab_old/tt_encoder.hip
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DTT_TIMING_BUILD -I$PWD -x hip -c"
/opt/rocm/bin/hipcc $F /tmp/ab_old/tt_encoder.hip -o ../build/variants/enc_o.o &
/opt/rocm/bin/hipcc $F tt_encoder.hip -o ../build/variants/enc_n.o &
wait
others=$(ls ../build/*.o | grep -v "tt_encoder")
for v in o n; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $others ../build/variants/enc_$v.o -o ../lib/variants/lib_$v.so
done
ls ../lib/variants

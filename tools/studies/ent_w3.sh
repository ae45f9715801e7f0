#!/usr/bin/env bash
# Study build of libaimet_amd.so whose entropy search kernel has no waves-per-EU hint (137 VGPRs,
# 4 workgroups per CU), to time against the product's (5 per CU):
#   bash tools/studies/ent_w3.sh && python tools/studies/tfe_search_time.py --lib tools/studies/ent_lib/w3/libaimet_amd.so ENTROPY
set -e
cd "$(dirname "$0")/../.."
make -C aimet_amd/csrc -j8 >/dev/null
SRC=aimet_amd/csrc/entropy_search.hip
FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Iinclude -Iaimet_amd/csrc --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-rdc"
SRCS=$(sed -n 's/^SRCS_\(HIP\|CPP\) = //p' aimet_amd/csrc/Makefile)
OBJS=$(for f in $SRCS; do b=${f%.*}; [ $b = entropy_search ] || echo build/obj/$b.o; done)
mkdir -p build/ent_variants tools/studies/ent_lib/w3
out=build/ent_variants/entropy_search_w3.hip
sed 's/ __attribute__((amdgpu_waves_per_eu(4)))//' $SRC > $out
grep -q amdgpu_waves_per_eu $out && { echo "hint not removed"; exit 1; }
/opt/rocm/bin/hipcc $FLAGS -x hip -c $out -o build/ent_variants/entropy_search_w3.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -Wl,--no-undefined -o tools/studies/ent_lib/w3/libaimet_amd.so $OBJS build/ent_variants/entropy_search_w3.o -lpthread
ls -la tools/studies/ent_lib/w3/libaimet_amd.so

#!/usr/bin/env bash
# Study builds of libaimet_amd.so for the MSE search:
#   tools/studies/mse_lib/nocand/libaimet_amd.so -- evaluates no candidate (each workgroup only loads
#     the channel's PDF, runs the setup and compacts the bins): the time of that preamble
#   tools/studies/mse_lib/w6/libaimet_amd.so     -- the search kernels at 6 waves per SIMD (80 VGPRs,
#     a few spills) instead of 5
#   bash tools/studies/mse_variants.sh && python tools/studies/tfe_search_time.py --lib tools/studies/mse_lib/nocand/libaimet_amd.so MSE
set -e
cd "$(dirname "$0")/../.."
make -C aimet_amd/csrc -j8 >/dev/null
SRC=aimet_amd/csrc/mse_search.hip
FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Iinclude -Iaimet_amd/csrc --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-rdc"
SRCS=$(sed -n 's/^SRCS_\(HIP\|CPP\) = //p' aimet_amd/csrc/Makefile)
OBJS=$(for f in $SRCS; do b=${f%.*}; [ $b = mse_search ] || echo build/obj/$b.o; done)
mkdir -p build/mse_variants tools/studies/mse_lib/nocand
out=build/mse_variants/mse_search_nocand.hip
sed 's/const long long j1    = j0 + chunk < full ? j0 + chunk : full;/const long long j1 = j0; (void) chunk; (void) full;/' $SRC > $out
grep -q "const long long j1 = j0;" $out || { echo "candidate range not replaced"; exit 1; }
/opt/rocm/bin/hipcc $FLAGS -x hip -c $out -o build/mse_variants/mse_search_nocand.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -Wl,--no-undefined -o tools/studies/mse_lib/nocand/libaimet_amd.so $OBJS build/mse_variants/mse_search_nocand.o -lpthread
mkdir -p tools/studies/mse_lib/w6
sed 's/amdgpu_waves_per_eu(5)/amdgpu_waves_per_eu(6)/g' $SRC > build/mse_variants/mse_search_w6.hip
grep -q "amdgpu_waves_per_eu(6)" build/mse_variants/mse_search_w6.hip || { echo "hint not replaced"; exit 1; }
/opt/rocm/bin/hipcc $FLAGS -x hip -c build/mse_variants/mse_search_w6.hip -o build/mse_variants/mse_search_w6.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -Wl,--no-undefined -o tools/studies/mse_lib/w6/libaimet_amd.so $OBJS build/mse_variants/mse_search_w6.o -lpthread
ls -la tools/studies/mse_lib/*/libaimet_amd.so

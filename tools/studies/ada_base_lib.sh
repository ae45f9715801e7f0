#!/usr/bin/env bash
# Study build of libaimet_amd.so with adaround.hip (and fast_pow.hpp) as of git revision $1
# (default HEAD), every other object the working tree's: an A/B baseline for a change under test.
#   bash tools/studies/ada_base_lib.sh [REV] && python tools/studies/ada_bwd_tune.py --lib tools/studies/ada_lib/base/libaimet_amd.so
set -e
cd "$(dirname "$0")/../.."
REV=${1:-HEAD}
make -C aimet_amd/csrc -j8 >/dev/null
FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Iinclude -Ibuild/ada_base -Iaimet_amd/csrc --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-rdc"
SRCS=$(sed -n 's/^SRCS_\(HIP\|CPP\) = //p' aimet_amd/csrc/Makefile)
OBJS=$(for f in $SRCS; do b=${f%.*}; [ $b = adaround ] || echo build/obj/$b.o; done)
mkdir -p build/ada_base tools/studies/ada_lib/base
git show $REV:aimet_amd/csrc/adaround.hip > build/ada_base/adaround.hip
git show $REV:aimet_amd/csrc/fast_pow.hpp > build/ada_base/fast_pow.hpp
/opt/rocm/bin/hipcc $FLAGS -x hip -c build/ada_base/adaround.hip -o build/ada_base/adaround.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -Wl,--no-undefined -o tools/studies/ada_lib/base/libaimet_amd.so $OBJS build/ada_base/adaround.o -lpthread
ls -la tools/studies/ada_lib/base/libaimet_amd.so

#!/usr/bin/env bash
# Study builds of libaimet_amd.so with the AdaRound backward's fast pow altered (timing only: the
# results are wrong by construction), to see where the pow's time goes:
#   tools/studies/ada_lib/nolds/libaimet_amd.so  -- the five LDS table reads per pow replaced by
#                                                   arithmetic on the index (same VALU shape)
#   tools/studies/ada_lib/nobar/libaimet_amd.so  -- no workgroup barrier after the table fill
# adaround.hip / fast_pow.hpp are edited by sed into build/ada_variants/<v>/; every other object
# is the product's (build/obj).
set -e
cd "$(dirname "$0")/../.."
make -C aimet_amd/csrc -j8 >/dev/null
FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Iinclude -Iaimet_amd/csrc --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-rdc"
SRCS=$(sed -n 's/^SRCS_\(HIP\|CPP\) = //p' aimet_amd/csrc/Makefile)
OBJS=$(for f in $SRCS; do b=${f%.*}; [ $b = adaround ] || echo build/obj/$b.o; done)
for v in nolds nobar; do
  d=build/ada_variants/$v
  mkdir -p $d
  cp aimet_amd/csrc/adaround.hip aimet_amd/csrc/fast_pow.hpp $d/
  if [ $v = nolds ]; then
    sed -i 's/g_pow_tab\.c\[j\]/(1.0f + (float) j * 0x1p-9f)/; s/g_pow_tab\.th\[j\]/((float) j * 0x1p-17f)/; s/g_pow_tab\.tl\[j\]/((float) j * 0x1p-40f)/; s/g_pow_tab\.eh\[i\]/(1.0f + (float) i * 0x1p-6f)/; s/g_pow_tab\.el\[i\]/((float) i * 0x1p-30f)/' $d/fast_pow.hpp
    grep -q "g_pow_tab\.\(c\|th\|tl\|eh\|el\)\[" $d/fast_pow.hpp && { echo "table read left"; exit 1; }
  else
    python3 - $d/adaround.hip <<'PY'
import sys
p = sys.argv[1]
s = open(p).read()
old = "            pow_tab_store<kBlock>(tab);\n            __syncthreads();\n            first = false;"
assert old in s
s = s.replace(old, "            pow_tab_store<kBlock>(tab);\n            first = false;")
open(p, "w").write(s)
PY
  fi
  /opt/rocm/bin/hipcc $FLAGS -x hip -c $d/adaround.hip -o $d/adaround.o
  mkdir -p tools/studies/ada_lib/$v
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -Wl,--no-undefined -o tools/studies/ada_lib/$v/libaimet_amd.so $OBJS $d/adaround.o -lpthread
done
ls -la tools/studies/ada_lib/*/libaimet_amd.so

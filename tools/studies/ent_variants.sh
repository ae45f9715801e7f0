#!/usr/bin/env bash
# Study builds of libaimet_amd.so whose entropy search skips steps (where its time goes):
#   tools/studies/ent_lib/no3/libaimet_amd.so  -- step 3 (the divergences) skipped
#   tools/studies/ent_lib/no23/libaimet_amd.so -- steps 2 and 3 skipped
#   tools/studies/ent_lib/no23w/libaimet_amd.so -- steps 2 and 3 skipped, and every window list the
#                                                 symmetric one (no asymmetric walk)
#   tools/studies/ent_lib/fw/, no23fw/           -- the asymmetric list from ent_walk_variant.py's walk
# The entropy source is edited by sed into build/ent_variants/; every other object is the
# product's (build/obj). Results are wrong by construction: timing / counters only.
#   bash tools/studies/ent_variants.sh && python tools/studies/tfe_search_time.py --lib tools/studies/ent_lib/no3/libaimet_amd.so ENTROPY
set -e
cd "$(dirname "$0")/../.."
make -C aimet_amd/csrc -j8 >/dev/null
SRC=aimet_amd/csrc/entropy_search.hip
FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Iinclude -Iaimet_amd/csrc --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-rdc"
# the product's objects (the Makefile's source lists; build/obj may hold stale ones)
SRCS=$(sed -n 's/^SRCS_\(HIP\|CPP\) = //p' aimet_amd/csrc/Makefile)
OBJS=$(for f in $SRCS; do b=${f%.*}; [ $b = entropy_search ] || echo build/obj/$b.o; done)
mkdir -p build/ent_variants
python3 tools/studies/ent_walk_variant.py $SRC build/ent_variants/entropy_search_fwsrc.hip
for v in no3 no23 no23w fw no23fw; do
  out=build/ent_variants/entropy_search_$v.hip
  src=$SRC
  case $v in *fw) src=build/ent_variants/entropy_search_fwsrc.hip;; esac
  if [ $v = fw ]; then cp $src $out; else
  sed 's/window_segment(hist, wa\[w\], wb\[w\], q0, q1, ws\[w\], pre, integral, dv, mag);/(void) q0; (void) q1;/' $src > $out
  fi
  if [ $v != no3 ] && [ $v != fw ]; then
    sed -i 's/window_norms_integral(hist, wa\[t\], wb\[t\], pre, ws\[t\], est);/ws[t].brk = 0;/' $out
  fi
  if [ $v = no23w ]; then
    sed -i -e 's/if (sym || strict)   \/\/ both ends/if (true)   \/\/ both ends/' -e 's/(sym || strict) ? entropy::kWindows/true ? entropy::kWindows/' $out
    grep -q "if (true)   // both ends" $out || { echo "window list not replaced"; exit 1; }
  fi
  [ $v = fw ] || ! grep -q "window_segment(hist, wa" $out || { echo "step 3 call not replaced"; exit 1; }
  /opt/rocm/bin/hipcc $FLAGS -x hip -c $out -o build/ent_variants/entropy_search_$v.o
  mkdir -p tools/studies/ent_lib/$v
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -Wl,--no-undefined -o tools/studies/ent_lib/$v/libaimet_amd.so $OBJS build/ent_variants/entropy_search_$v.o -lpthread
done
ls -la tools/studies/ent_lib/*/libaimet_amd.so

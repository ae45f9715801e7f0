#!/usr/bin/env bash
# Round 6, session x: the strided-block QDQ kernel with row groups rotated per block (study builds),
# alternating with the round-5 form.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
L=tools/studies/bcast_lib
k=0
for v in base r64b4t0 r64b4t1 r64b8t1 r32b4t1 r64b2t1 base r64b4t0 r64b4t1; do
  k=$((k+1))
  run bc${k}_$v 120 python tools/studies/bcast_tune.py --lib $L/$v/libaimet_amd.so --tag $v
done

#!/usr/bin/env bash
# Round 6, session w: the strided-block QDQ kernel -- whole-block rows, encodings after the first
# rows' loads, next group prefetched -- against the round-5 form (study builds), then parity.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
L=tools/studies/bcast_lib
for v in base r16b8 r32b8 r64b4 r64b8 r64b16 base r64b8; do
  run bc_$v 120 python tools/studies/bcast_tune.py --lib $L/$v/libaimet_amd.so --tag $v
done
run t_bc 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_blockwise.py

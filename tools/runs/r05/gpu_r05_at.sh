#!/usr/bin/env bash
# Round 5, session at: the AdaRound backward at 2^28 with 64 vs 4096 channels on one box (session as
# measured 64 channels at 1.13 ms against 1.23-1.33 for 4096 on other boxes): box or shape?
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
for C in 64 4096 64 4096 1; do
  run ada_ch_$C 300 python -u tools/studies/ada_bwd_tune.py --scales 1 --channels $C --tag ch$C
  grep -h '^{' $OUT/ada_ch_$C.log >> $OUT/ada_bwd_channels.jsonl
done

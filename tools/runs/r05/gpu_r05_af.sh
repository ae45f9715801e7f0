#!/usr/bin/env bash
# Round 5, session af: the parameters' per-channel statistics kernels (channel_minmax_fold_many,
# channel_hist_fold_many; one workgroup per channel, 27,560 channels) held to 2 / 4 / 8 workgroups
# per CU beside the activations' min/max pass -- temporary builds (dynamic-LDS padding), removed
# after; tools/studies/enc_plan_runs.py, form both, alternating with the unpadded build.
# Result (profiles/r05/enc_stats_cap.jsonl): uncapped 3.63 / 3.69 ms; 2 per CU 4.14, 4 per CU 3.81,
# 8 per CU 3.72 -- the statistics then delay the parameters' search behind them. Not adopted.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
for L in scu0 scu2 scu4 scu8 scu0 scu4; do
  run enc_$L 240 python -u tools/studies/enc_plan_runs.py --reps 30 --forms both --lib tools/studies/exp_libs/lib_$L.so --tag $L
  grep -h '^{' $OUT/enc_$L.log >> $OUT/enc_stats_cap.jsonl
done

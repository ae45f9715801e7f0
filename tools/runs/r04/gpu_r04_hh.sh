#!/usr/bin/env bash
# Round 4, session hh: the weights' TF-E search with a capped grid (AIMET_TUNE_TFE_GRID: fewer of its
# workgroups resident beside the activations' min/max pass) -- compute_encodings medians.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run enc_split_default 300 python -u tools/studies/enc_split_cost.py --reps 11
for g in 256 512 1024 2048; do
  AIMET_TUNE_TFE_GRID=$g run enc_split_g$g 300 python -u tools/studies/enc_split_cost.py --reps 11
done

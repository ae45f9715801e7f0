#!/usr/bin/env bash
# Round 3: compute_encodings schedule -- the parameters' search beside the min/max pass (default)
# or the histogram pass, TF-E grid caps. A/B/A order, 2 runs each.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
for rep in 1 2; do
  for cfg in "0 0" "1 0" "0 1024" "1 1024" "1 512"; do
    set -- $cfg
    run ce_${1}_${2}_$rep 200 env AIMET_CAL_PAR_SEARCH=$1 AIMET_TUNE_TFE_GRID=$2 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline
  done
done

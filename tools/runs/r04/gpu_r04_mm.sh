#!/usr/bin/env bash
# Round 4, session mm: the parameters' statistics and search beside the histogram pass instead of the
# min/max pass (AIMET_CAL_PARAMS_AFTER_MINMAX=1: a study switch in quantizer.cpp, removed after this
# run measured it slower) -- compute_encodings medians and bench lines.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run enc_default 300 python -u tools/studies/enc_split_cost.py --reps 11
AIMET_CAL_PARAMS_AFTER_MINMAX=1 run enc_after 300 python -u tools/studies/enc_split_cost.py --reps 11
run bench_default 300 python -u bench.py --no-cpu-baseline
AIMET_CAL_PARAMS_AFTER_MINMAX=1 run bench_after 300 python -u bench.py --no-cpu-baseline
run bench_default2 300 python -u bench.py --no-cpu-baseline
AIMET_CAL_PARAMS_AFTER_MINMAX=1 run bench_after2 300 python -u bench.py --no-cpu-baseline
AIMET_CAL_PARAMS_AFTER_MINMAX=1 run t_cal 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "calib or encoding or tfe"

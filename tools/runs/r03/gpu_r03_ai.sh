#!/usr/bin/env bash
# Round 3: aimet_adaround_dw_step variants (positions in flight per lane, positions per slice).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run dwt_def 120 python -u tools/studies/dw_step_tune.py default
run dwt_u1 120 env AIMET_TUNE_DW_U=1 python -u tools/studies/dw_step_tune.py u1
run dwt_u2 120 env AIMET_TUNE_DW_U=2 python -u tools/studies/dw_step_tune.py u2
run dwt_u8 120 env AIMET_TUNE_DW_U=8 python -u tools/studies/dw_step_tune.py u8
run dwt_p4 120 env AIMET_TUNE_DW_PER=4 python -u tools/studies/dw_step_tune.py per4
run dwt_p8 120 env AIMET_TUNE_DW_PER=8 python -u tools/studies/dw_step_tune.py per8
run dwt_p32 120 env AIMET_TUNE_DW_PER=32 python -u tools/studies/dw_step_tune.py per32
run dwt_p8u8 120 env AIMET_TUNE_DW_PER=8 AIMET_TUNE_DW_U=8 python -u tools/studies/dw_step_tune.py per8u8
cat $OUT/dwt_*.log | grep '^{' > $OUT/dw_step_tune.jsonl

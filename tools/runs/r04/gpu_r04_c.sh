#!/usr/bin/env bash
# Round 4, session c: checkpoint tests with deterministic MIOpen; Llama range-gradient units measured.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
export AIMET_BOUND_REPORT=$OUT/lg_bound_units_llama.jsonl
rm -f $AIMET_BOUND_REPORT
run t_ckpt 600 python -u -m pytest tests/test_checkpoint.py -v --timeout 300 --timeout-method thread
AIMET_LG_BOUND_C=64 run t_llama 600 python -u -m pytest tests/test_llama_quantsim_gpu.py -v --timeout 300 --timeout-method thread

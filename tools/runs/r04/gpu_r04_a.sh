#!/usr/bin/env bash
# Round 4, session a: checkpoint / resume, RCCL world-1 exchange, non-contiguous calibration inputs,
# few-output-channel pointwise step, learned-grid range-gradient error measured in bound units.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
export AIMET_BOUND_REPORT=$OUT/lg_bound_units.jsonl
rm -f $AIMET_BOUND_REPORT
run t_ckpt 600 python -u -m pytest tests/test_checkpoint.py tests/test_distributed_gpu.py -v --timeout 300 --timeout-method thread
run t_parity 600 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "calibrate or pw_step or learned_grid_vs_reference_golden or learned_grid_large"
run t_llama 600 python -u -m pytest tests/test_llama_quantsim_gpu.py -v --timeout 300 --timeout-method thread

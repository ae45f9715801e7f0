#!/usr/bin/env bash
# Round 5, session ae: learned-grid per-channel initialisation from arrays -- the range-learning /
# Llama QuantSim / checkpoint / DDP tests, and config 5's calibration profiled again.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_rl 900 python -u -m pytest tests/test_range_learning.py tests/test_llama_quantsim_gpu.py tests/test_checkpoint.py tests/test_qat_ddp_gpu.py -q --timeout 600 --timeout-method thread -m gpu
run llama_prof 900 python -u benchmarks/llama_qat.py --steps 2 --warmup 1 --profile-calib

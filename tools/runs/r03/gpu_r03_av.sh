#!/usr/bin/env bash
# Round 3: config 5's 2-layer Llama QuantSim forward vs the reference's torch ops (bf16 autocast).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run llama_qs 600 python -u -m pytest tests/test_llama_quantsim_gpu.py tests/test_gpu_parity.py -k "llama or calibrate" -m gpu -x -v --timeout 300 --timeout-method thread

#!/usr/bin/env bash
# Round 5, session aa: config 5's QuantizationSimModel.compute_encodings profiled (2 steps after).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run llama_prof 900 python -u benchmarks/llama_qat.py --steps 2 --warmup 1 --profile-calib

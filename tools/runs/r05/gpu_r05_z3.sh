#!/usr/bin/env bash
# Round 5, session z3: config 1's oracle test recording the tensors handed to the StatsBatch.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_c1 600 python -u -m pytest tests/test_configs_gpu.py -v --timeout 600 --timeout-method thread -k "config1"

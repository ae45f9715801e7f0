#!/usr/bin/env bash
# Round 5, session r: config 4's sharded calibration test with the calibration plan's staged launch
# (318 quantizers over a 2-rank gloo group) beside the phased form.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_vit 900 python -u -m pytest tests/test_configs_gpu.py -v --timeout 600 --timeout-method thread -k "config4"

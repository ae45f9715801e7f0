#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_gelu 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py -k "fused_step"
run cfg1_cpu 900 python -u benchmarks/resnet_quantsim.py --cpu-model
echo ALLDONE

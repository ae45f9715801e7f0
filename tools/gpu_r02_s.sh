#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_cal 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_configs_gpu.py -k "calibrate or resident or reset or config1 or bench"
run tune 600 python -u tools/enc_partition_tune.py params_first:0 params_first_phased:0 params_first:0
run bench 300 python bench.py
echo ALLDONE

#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_reset 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_configs_gpu.py -k "reset or bench or many"
run sched 500 python tools/enc_schedule_tune.py
run bench 300 python bench.py --no-cpu-baseline
echo ALLDONE

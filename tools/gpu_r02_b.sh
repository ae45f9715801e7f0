#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_new 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_range_learning.py tests/test_dropin_boundary.py
run t_vit 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_configs_gpu.py -k config4
run vit_bench 400 python benchmarks/vit_calibration.py
run ada_prof 400 rocprofv3 --kernel-trace --stats -d "$OUT/ada_prof" -o run --output-format csv -- python3 benchmarks/adaround_mobilenet.py --iterations 500
rm -f "$OUT"/ada_prof/*kernel_trace.csv
echo ALLDONE

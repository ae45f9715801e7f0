#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_new 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_range_learning.py tests/test_dropin_boundary.py
run llama_qs 600 python benchmarks/llama_qat.py --layers 32 --steps 5 --warmup 2
run ada_prof 400 rocprofv3 --kernel-trace --stats -d "$OUT/ada_prof" -o run --output-format csv -- python3 benchmarks/adaround_mobilenet.py --iterations 500
echo ALLDONE

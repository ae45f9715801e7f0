#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_ada 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_adaround_golden.py tests/test_adaround_dist_gpu.py -k "adaround or recon or depthwise"
run ada_warm 300 python -u benchmarks/adaround_mobilenet.py --iterations 300
run ada_10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000 --reference-iters 300
echo ALLDONE

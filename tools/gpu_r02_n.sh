#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_ada 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_adaround_golden.py tests/test_adaround_dist_gpu.py -k "adaround or recon or depthwise"
run ada_gemm 300 python benchmarks/adaround_mobilenet.py --iterations 500
AIMET_ADA_GEMM_LAYERS=0 run ada_nogemm 300 python benchmarks/adaround_mobilenet.py --iterations 500
run ceiling 200 python tools/read_ceiling.py
echo ALLDONE

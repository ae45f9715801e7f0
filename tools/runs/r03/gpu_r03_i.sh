#!/usr/bin/env bash
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ddp 900 python -u -m pytest tests/test_qat_ddp_gpu.py -q -s --timeout 800 --timeout-method thread
run vit 300 python -u benchmarks/vit_calibration.py --images 160 --oracle-check 0
run stats_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "histogram or hist or minmax or stats or config or calibration or entropy or boundary or many"

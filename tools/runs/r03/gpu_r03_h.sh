#!/usr/bin/env bash
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run san 300 python -u -m pytest tests/test_sanitize.py -m gpu -x -q --timeout 250 --timeout-method thread
run ddp 900 python -u -m pytest tests/test_qat_ddp_gpu.py -x -q --timeout 800 --timeout-method thread
run vit 300 python -u benchmarks/vit_calibration.py --images 160 --oracle-check 0

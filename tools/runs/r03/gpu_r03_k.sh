#!/usr/bin/env bash
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run vit 300 python -u benchmarks/vit_calibration.py --images 160 --oracle-check 0
run gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run bench 600 python -u bench.py

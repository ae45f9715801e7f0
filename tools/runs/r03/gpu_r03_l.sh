#!/usr/bin/env bash
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run vit 300 python -u benchmarks/vit_calibration.py --images 160 --oracle-check 0
run vit_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/vit_trace -o run -- python3 benchmarks/vit_calibration.py --images 96 --oracle-check 0

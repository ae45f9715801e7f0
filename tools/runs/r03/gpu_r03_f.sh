#!/usr/bin/env bash
# Round 3: tile-form per-tensor learned-grid kernels, chunking past 2^31.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run lg_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "learned or lg or range_learning or qat"
run lg16_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/lg16_trace -o run -- python3 benchmarks/lg16_roofline.py --reps 20

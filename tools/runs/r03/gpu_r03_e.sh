#!/usr/bin/env bash
# Round 3: learned-grid quotients by one Markstein correction + ViT split.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run lg_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "learned or lg or range_learning or qat"
run lg16 300 python -u benchmarks/lg16_roofline.py
run lg16_b8 300 python -u benchmarks/lg16_roofline.py --bitwidth 8
run kr 300 python -u benchmarks/kernel_roofline.py --no-cpu --reps 10
run vit 300 python -u benchmarks/vit_calibration.py --images 160 --oracle-check 0
run lg16_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/lg16_trace -o run -- python3 benchmarks/lg16_roofline.py --reps 20

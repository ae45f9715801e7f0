#!/usr/bin/env bash
# Round 3: AdaRound pow shortcuts (exact) + loss-free gradient path; kernel roofline and loop.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "adaround"
run kr 300 python -u benchmarks/kernel_roofline.py --no-cpu --reps 10
run ada2k 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000

#!/usr/bin/env bash
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "adaround"
run ada_div 900 python -u tools/studies/adaround_loop_divergence.py
run ada_mnv2 900 python -u benchmarks/adaround_mobilenet.py --iterations 2000

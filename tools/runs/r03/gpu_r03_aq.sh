#!/usr/bin/env bash
# Round 3: quad forms (stride 1) of the depthwise weight gradient and one-pass step; bit-identity tests, timings, config 3.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_adaround_wrapper.py -m gpu -x -q --timeout 300 --timeout-method thread -k "dw or depthwise or adaround_loop"
grep -q " passed" $OUT/ada_tests.log && ! grep -q "failed\|error" $OUT/ada_tests.log || { echo "tests failed"; exit 1; }
run dwt_quad 120 python -u tools/studies/dw_step_tune.py quad
run ada10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000

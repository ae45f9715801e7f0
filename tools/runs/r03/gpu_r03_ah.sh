#!/usr/bin/env bash
# Round 3: the one-pass 1x1 form by shape rule (expanding layers at >= 56^2); AdaRound tests + config 3.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_adaround_wrapper.py tests/test_adaround_golden.py -m gpu -x -q --timeout 300 --timeout-method thread -k "adaround or dw or depthwise or pw_step"
grep -q " passed" $OUT/ada_tests.log && ! grep -q "failed\|error" $OUT/ada_tests.log || { echo "tests failed"; exit 1; }
run ada10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000

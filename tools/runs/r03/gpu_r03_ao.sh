#!/usr/bin/env bash
# Round 3: the pointwise step with position-major LDS images; parity tests, config 3 with every
# eligible 1x1 layer one-pass (AIMET_ADA_PW_FUSED=all) to re-measure the per-layer forms.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_adaround_wrapper.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pw_step or pw_fused or adaround_loop_deterministic"
grep -q " passed" $OUT/ada_tests.log && ! grep -q "failed\|error" $OUT/ada_tests.log || { echo "tests failed"; exit 1; }
run ada10k_all 900 env AIMET_ADA_PW_FUSED=all python -u benchmarks/adaround_mobilenet.py --iterations 10000

#!/usr/bin/env bash
# Round 3: the LDS-staged depthwise step; bit-identity tests, the variant timings, config 3.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_adaround_wrapper.py -m gpu -x -q --timeout 300 --timeout-method thread -k "dw or depthwise"
grep -q " passed" $OUT/ada_tests.log && ! grep -q "failed\|error" $OUT/ada_tests.log || { echo "tests failed"; exit 1; }
run dwt_lds 120 python -u tools/studies/dw_step_tune.py lds
run dwt_nolds 120 env AIMET_TUNE_DW_LDS=0 python -u tools/studies/dw_step_tune.py global
cat $OUT/dwt_lds.log $OUT/dwt_nolds.log | grep '^{' > $OUT/dw_step_lds.jsonl
run ada10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000

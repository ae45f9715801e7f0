#!/usr/bin/env bash
# Round 3: the activations' min/max pass enqueued first (resets and the parameters' work after it);
# calibration tests, bench x3, a kernel trace of the bench.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ce_tests 600 python -u -m pytest tests/test_configs_gpu.py tests/test_gpu_parity.py tests/test_sanitize.py -m gpu -x -q --timeout 300 --timeout-method thread
grep -q " passed" $OUT/ce_tests.log && ! grep -q "failed\|error" $OUT/ce_tests.log || { echo "tests failed"; exit 1; }
for rep in 1 2 3; do
  run ce_r$rep 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline
done
run ce_trace 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/ce_trace4 -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline

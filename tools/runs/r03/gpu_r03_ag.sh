#!/usr/bin/env bash
# Round 3: fused depthwise step with positions in flight + the fused 1x1 step (aimet_adaround_pw_step);
# parity tests, then config 3 and a kernel trace of a short run (summarised on the box, raw trace dropped).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_adaround_wrapper.py tests/test_adaround_golden.py -m gpu -x -q --timeout 300 --timeout-method thread -k "adaround or dw or depthwise or pw_step"
grep -q " passed" $OUT/ada_tests.log && ! grep -q "failed\|error" $OUT/ada_tests.log || { echo "tests failed"; exit 1; }
run ada10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000
run ada_trace 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/ada_trace -o run -- python3 benchmarks/adaround_mobilenet.py --iterations 100
python tools/studies/ada_trace_summary.py $OUT/ada_trace 5300 $OUT/ada_loop_kernels.csv > $OUT/ada_loop_summary.txt 2>&1
rm -rf $OUT/ada_trace

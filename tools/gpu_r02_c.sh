#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_new 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_range_learning.py tests/test_dropin_boundary.py tests/test_gpu_parity.py -k "learned or range or dropin or staged or replica or cpu"
run t_vit 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_configs_gpu.py -k config4
run ada_base 300 python benchmarks/adaround_mobilenet.py --iterations 500
run ada_find 300 python benchmarks/adaround_mobilenet.py --iterations 500 --miopen-find
run ada_prof 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/ada_prof2" -o run -- python3 benchmarks/adaround_mobilenet.py --iterations 200 --miopen-find
run ada_sum 120 python tools/ada_trace_summary.py "$OUT/ada_prof2" 10600 "$OUT/ada_loop_kernels.csv"
rm -f "$OUT"/ada_prof2/*kernel_trace.csv
echo ALLDONE

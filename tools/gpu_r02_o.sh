#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_ada 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_adaround_golden.py tests/test_adaround_dist_gpu.py -k "adaround or recon or depthwise"
run ada_500 300 python benchmarks/adaround_mobilenet.py --iterations 500
run ada_prof 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/ada_prof5" -o run -- python3 benchmarks/adaround_mobilenet.py --iterations 200
run ada_sum 120 python tools/ada_trace_summary.py "$OUT/ada_prof5" 10600 "$OUT/ada_loop_kernels.csv"
rm -f "$OUT"/ada_prof5/*kernel_trace.csv
run ada_10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000 --reference-iters 300
echo ALLDONE

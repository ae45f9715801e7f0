#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run ceiling 200 python tools/read_ceiling.py
run ada_prof 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/ada_prof4" -o run -- python3 benchmarks/adaround_mobilenet.py --iterations 200
run ada_sum 120 python tools/ada_trace_summary.py "$OUT/ada_prof4" 10600 "$OUT/ada_loop_kernels.csv"
rm -f "$OUT"/ada_prof4/*kernel_trace.csv
run ada_10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000 --reference-iters 300
echo ALLDONE

#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run prof_enc 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/prof_enc" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
run tl 60 python tools/trace_timeline.py "$OUT/prof_enc/run_kernel_trace.csv" minmax_many_kernel 30 40
run mc 60 python tools/copy_timeline.py "$OUT/prof_enc" minmax_many_kernel
rm -f "$OUT"/prof_enc/*trace.csv
echo ALLDONE

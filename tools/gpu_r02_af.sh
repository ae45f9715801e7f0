#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run plain_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/lpp" -o run -- python3 benchmarks/llama_qat.py --path plain --layers 32 --steps 3 --warmup 1
rm -f "$OUT"/lpp/*kernel_trace.csv
echo ALLDONE

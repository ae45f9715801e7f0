#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run pk 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pk" -o run -- python3 tools/pass_kernel_times.py
rm -f "$OUT"/pk/*kernel_trace.csv
echo ALLDONE

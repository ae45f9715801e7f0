#!/usr/bin/env bash
# Round 4 closing check D: rocprofv3 --kernel-trace --stats of the bench command (per-kernel average
# durations behind the bench line's roofline).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run bench_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench_stats -o run -- python3 bench.py --steps 20 --no-cpu-baseline
python tools/studies/prof_summary.py $OUT/bench_stats --steps 20 > $OUT/bench_stats_summary.txt 2>&1
rm -f $OUT/bench_stats/run_kernel_trace.csv

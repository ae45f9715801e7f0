#!/usr/bin/env bash
# Round 3: compute_encodings two native calls vs one, interleaved (40 reps each); the bench line
# and its kernel trace at this commit.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run enc_ab 300 python -u tools/studies/enc_split_ab.py 40
run bench 300 python -u bench.py
run bench_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench_trace -o run -- python3 bench.py --steps 20 --no-cpu-baseline
python tools/studies/prof_summary.py $OUT/bench_trace --steps 20 > $OUT/bench_trace_summary.txt 2>&1
rm -f $OUT/bench_trace/run_kernel_trace.csv

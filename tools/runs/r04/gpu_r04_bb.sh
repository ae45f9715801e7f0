#!/usr/bin/env bash
# Round 4, session bb: the weights' TF-E search without register spills (128-lane form at 4 waves
# per SIMD: 111 VGPRs, no scratch; it spilled 28 B per lane at 5) -- the TF-E / calibration tests,
# the bench line with the CPU compute_encodings baseline measured on the whole batch (no
# projection), and the bench's kernel stats.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_tfe 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "tfe or calib or encoding"
run bench 900 python -u bench.py
run bench_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench_stats -o run -- python3 bench.py --steps 20 --no-cpu-baseline
python tools/studies/prof_summary.py $OUT/bench_stats --steps 20 > $OUT/bench_stats_summary.txt 2>&1
rm -f $OUT/bench_stats/run_kernel_trace.csv

#!/usr/bin/env bash
# Round 4, session x: one compute_encodings call's kernel timeline (critical path and launch gaps,
# tools/studies/enc_timeline.py) and the kernel rooflines at the new AdaRound backward.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run enc_trace 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/enc_trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
python3 tools/studies/enc_timeline.py $OUT/enc_trace > $OUT/enc_timeline.txt 2>&1
rm -rf $OUT/enc_trace
run roofline 600 python -u benchmarks/kernel_roofline.py

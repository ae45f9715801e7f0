#!/usr/bin/env bash
# Round 4, session y: one compute_encodings call's kernels and host HIP calls on one clock
# (rocprofv3 --kernel-trace --hip-runtime-trace; tools/studies/enc_timeline.py).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run enc_trace 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $OUT/enc_trace2 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
python3 tools/studies/enc_timeline.py $OUT/enc_trace2 > $OUT/enc_timeline_api.txt 2>&1
rm -rf $OUT/enc_trace2

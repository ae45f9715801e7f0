#!/usr/bin/env bash
# Round 4, session z: the activations' search job table uploaded on the parameters' stream (no copy
# between the last histogram fold and the search) -- calibration tests, two bench lines, the
# compute_encodings timeline again.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_cal 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "calib or encoding or tfe or quantsim or distributed or config"
run bench1 300 python -u bench.py --no-cpu-baseline
run bench2 300 python -u bench.py --no-cpu-baseline
run enc_trace 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $OUT/enc_trace3 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
python3 tools/studies/enc_timeline.py $OUT/enc_trace3 > $OUT/enc_timeline_api_z.txt 2>&1
rm -rf $OUT/enc_trace3

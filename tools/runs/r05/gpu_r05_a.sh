#!/usr/bin/env bash
# Round 5, session a: calibration plans (aimet_calib_plan_*) -- calibration / distributed tests, bench
# lines with the plan headline and the world-1 RCCL exchange, the compute_encodings timeline.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_cal 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "calib or encoding or resident or distributed or bench_calibration or reset_of"
run bench1 300 python -u bench.py --no-cpu-baseline --force-exchange
run bench2 300 python -u bench.py --no-cpu-baseline
run enc_trace 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $OUT/enc_trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
python3 tools/studies/enc_timeline.py $OUT/enc_trace > $OUT/enc_timeline_plan.txt 2>&1
rm -rf $OUT/enc_trace

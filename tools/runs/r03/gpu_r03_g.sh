#!/usr/bin/env bash
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run lg_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "learned or lg or range_learning or qat"
for v in 2 4; do
run lg16_trace_v$v 300 env AIMET_TUNE_LG16_VECS=$v rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/lg16_trace_v$v -o run -- python3 benchmarks/lg16_roofline.py --reps 20
done

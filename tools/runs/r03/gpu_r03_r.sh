#!/usr/bin/env bash
# Round 3: learned-grid 16-bit kernels -- instruction counts (PMC) + traces; lg tests.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run lg_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "learned or lg or range_learning or qat"
run lgt3 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/lgt3 -o run -- python3 benchmarks/lg16_roofline.py --reps 40
python3 tools/studies/lg16_trace_summary.py $OUT/lgt3 "fastpath" >> $OUT/lg_new.jsonl
run lgpmc 120 timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $OUT/lgpmc -o run -- python3 benchmarks/lg16_roofline.py --reps 5

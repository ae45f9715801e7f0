#!/usr/bin/env bash
# Round 3: learned-grid clamp-then-Markstein forward, per-mode backward kernels.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run lg_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "learned or lg or range_learning or qat"
for i in 1 2; do
  run lgu$i 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/lgu$i -o run -- python3 benchmarks/lg16_roofline.py --reps 40
  python3 tools/studies/lg16_trace_summary.py $OUT/lgu$i "modes$i" >> $OUT/lg_modes.jsonl
done
run lgpmc2 120 timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d $OUT/lgpmc2 -o run -- python3 benchmarks/lg16_roofline.py --reps 5

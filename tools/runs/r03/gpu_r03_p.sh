#!/usr/bin/env bash
# Round 3: reciprocal-Newton exhaustive check; learned-grid NaN semantics + branch-free forward;
# AdaRound with one Sleef logkf per element.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run rcp 120 ./tools/studies/rcp_newton_check
run lg_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "learned or lg or range_learning or qat"
run ada_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "adaround"
for i in 1 2; do
  run lgt$i 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/lgt$i -o run -- python3 benchmarks/lg16_roofline.py --reps 40
  python3 tools/studies/lg16_trace_summary.py $OUT/lgt$i "new$i" >> $OUT/lg_new.jsonl
done
run kr 300 python -u benchmarks/kernel_roofline.py --no-cpu --reps 10

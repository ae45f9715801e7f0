#!/usr/bin/env bash
# Round 3: software-pipelined 16-bit learned-grid kernels (shape sweep) + AdaRound reciprocal.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run lg_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "learned or lg or range_learning or qat"
run ada_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "adaround"
i=0
for cfg in "1:256:2048 2:2048" "2:256:1024 1:2048" "1:256:4096 2:1024" "2:256:2048 1:4096" "1:512:1024 2:4096" "1:256:2048 2:2048"; do
  set -- $cfg
  i=$((i+1))
  run lgp$i 200 env AIMET_TUNE_LG16_FWD=$1 AIMET_TUNE_LG_BWD=$2 rocprofv3 --kernel-trace --output-format csv -d $OUT/lgp$i -o run -- python3 benchmarks/lg16_roofline.py --reps 40
  python3 tools/studies/lg16_trace_summary.py $OUT/lgp$i "fwd=$1 bwd=$2" >> $OUT/lg_pipe.jsonl
done
run kr 300 python -u benchmarks/kernel_roofline.py --no-cpu --reps 10

#!/usr/bin/env bash
# Round 3: launch-shape variants of the 16-bit learned-grid kernels, then the
# AdaRound checks (wrapper, adaround_module, determinism, divergence study, MobileNet-v2 loop).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run lg_tests_loop 600 env AIMET_TUNE_LG_BWD=4:512 AIMET_TUNE_LG16_FWD=1:512:700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "learned_grid and (16 or chunk or tensor)"
i=0
for cfg in "2:256:0 2:0" "1:256:0 1:0" "4:256:0 4:0" "2:512:0 2:2048" "1:512:0 1:4096" "1:1024:0 4:1024" "2:1024:0 2:1024" "2:256:2048 1:2048" "1:256:4096 2:4096"; do
  set -- $cfg
  i=$((i+1))
  run lgv$i 200 env AIMET_TUNE_LG16_FWD=$1 AIMET_TUNE_LG_BWD=$2 rocprofv3 --kernel-trace --output-format csv -d $OUT/lgv$i -o run -- python3 benchmarks/lg16_roofline.py --reps 40
  python3 tools/studies/lg16_trace_summary.py $OUT/lgv$i "fwd=$1 bwd=$2" >> $OUT/lg_variants.jsonl
done
run ada_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "adaround"
run ada_div 900 python -u tools/studies/adaround_loop_divergence.py
run ada_mnv2 900 python -u benchmarks/adaround_mobilenet.py --iterations 2000

#!/usr/bin/env bash
# Round 3: launch shapes of the 16-bit learned-grid kernels after the VALU cuts.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
i=0
for cfg in "2:256:0 2:0" "4:256:0 1:0" "8:256:0 2:2048" "2:256:1024 2:1024" "4:256:1024 1:4096" "2:512:0 2:0" "4:256:2048 1:0" "2:256:0 2:0"; do
  set -- $cfg
  i=$((i+1))
  run lgs$i 200 env AIMET_TUNE_LG16_FWD=$1 AIMET_TUNE_LG_BWD=$2 rocprofv3 --kernel-trace --output-format csv -d $OUT/lgs$i -o run -- python3 benchmarks/lg16_roofline.py --reps 40
  python3 tools/studies/lg16_trace_summary.py $OUT/lgs$i "fwd=$1 bwd=$2" >> $OUT/lg_shapes.jsonl
done

#!/usr/bin/env bash
# Round 4, session k: where the AdaRound loop's time goes at k iterations per graph (kernel busy vs
# gaps), library vs MFMA channel-major step; LG16 backward with one group per lane below 4 M elements.
# The raw traces are summarised on the box and removed (the loop traces exceed the copy-back cap).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run lg16_trace 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lg16_trace -o run -- python3 benchmarks/lg16_roofline.py --reps 40
python tools/studies/lg16_trace_summary.py $OUT/lg16_trace r04 > $OUT/lg16_trace_summary.txt 2>&1
run ada_trace 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/ada_trace -o run -- python3 benchmarks/adaround_mobilenet.py --iterations 200
python tools/studies/ada_trace_summary.py $OUT/ada_trace $((53*200)) > $OUT/ada_trace_summary.txt 2>&1
rm -rf $OUT/ada_trace
AIMET_ADA_PW_CM_FUSED=1 run ada_trace_cm 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/ada_trace_cm -o run -- python3 benchmarks/adaround_mobilenet.py --iterations 200
python tools/studies/ada_trace_summary.py $OUT/ada_trace_cm $((53*200)) > $OUT/ada_trace_cm_summary.txt 2>&1
rm -rf $OUT/ada_trace_cm
run pw_cm_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/pw_cm_stats -o run -- python3 tools/studies/pw_cm_bench.py --reps 50
rm -f $OUT/pw_cm_stats/run_kernel_trace.csv

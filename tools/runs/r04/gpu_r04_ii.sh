#!/usr/bin/env bash
# Round 4, session ii: the trace of the loop config 3 ships at the final tree (the steps' slices
# added by the Adam step, the backward's tail flag, the 28 x 28 projecting-layer rule).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_trace 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/ada_trace -o run -- python3 benchmarks/adaround_mobilenet.py --iterations 200
python tools/studies/ada_trace_summary.py $OUT/ada_trace $((53*200)) > $OUT/ada_trace_summary.txt 2>&1
rm -rf $OUT/ada_trace

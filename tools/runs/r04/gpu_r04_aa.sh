#!/usr/bin/env bash
# Round 4, session aa: the per-tensor learned-grid backward with 4 eight-element groups per lane and
# tile (AIMET_TUNE_LG_BWD=4:0; half the tiles, so half the per-tile reductions and fold parts)
# against the default 2 -- kernel trace, and the range-gradient bound / equality tests under it.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run lg16_s2 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lg16_s2 -o run -- python3 benchmarks/lg16_roofline.py --reps 40
python tools/studies/lg16_trace_summary.py $OUT/lg16_s2 steps2 > $OUT/lg16_s2_summary.txt 2>&1
AIMET_TUNE_LG_BWD=4:0 run lg16_s4 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lg16_s4 -o run -- python3 benchmarks/lg16_roofline.py --reps 40
python tools/studies/lg16_trace_summary.py $OUT/lg16_s4 steps4 > $OUT/lg16_s4_summary.txt 2>&1
rm -f $OUT/lg16_s2/run_kernel_trace.csv $OUT/lg16_s4/run_kernel_trace.csv
AIMET_TUNE_LG_BWD=4:0 AIMET_BOUND_REPORT=$OUT/lg_bound_s4.jsonl run t_lg_s4 900 python -u -m pytest tests/test_gpu_parity.py tests/test_range_learning.py tests/test_llama_quantsim_gpu.py -q --timeout 300 --timeout-method thread -k "learned_grid or lg_ or range or llama"

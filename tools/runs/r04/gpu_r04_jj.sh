#!/usr/bin/env bash
# Round 4, session jj: the 16-bit learned-grid backward's asymmetric-mode kernel compiled for 4 waves
# per SIMD (library built with -DAIMET_LG_BWD16_MINW4: 128 VGPRs + a small spill instead of 134) --
# kernel trace and the learned-grid tests.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run lg16_w4 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lg16_w4 -o run -- python3 benchmarks/lg16_roofline.py --reps 40
python tools/studies/lg16_trace_summary.py $OUT/lg16_w4 minw4 > $OUT/lg16_w4_summary.txt 2>&1
rm -f $OUT/lg16_w4/run_kernel_trace.csv
run t_lg 900 python -u -m pytest tests/test_gpu_parity.py tests/test_range_learning.py -q --timeout 300 --timeout-method thread -k "learned_grid or lg_ or range"

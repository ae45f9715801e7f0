#!/usr/bin/env bash
# Round 5, session an: the AdaRound grid-forms test (with the round-loss value check), and a kernel
# trace of the 2^28 backward runs (reg 0.01 and reg 0) whose per-kernel averages must agree with
# the HIP-event timings of ada_bwd_tune.py.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_grid_test 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "grid_forms"
run ada_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ada_trace -o run -- python3 tools/studies/ada_bwd_tune.py --scales 1 --tag trace
run ada_trace0 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ada_trace0 -o run -- python3 tools/studies/ada_bwd_tune.py --scales 1 --reg 0 --tag trace_reg0
cp $OUT/ada_trace/run_kernel_stats.csv $OUT/ada_bwd_kernel_stats.csv 2>/dev/null
cp $OUT/ada_trace0/run_kernel_stats.csv $OUT/ada_bwd_kernel_stats_reg0.csv 2>/dev/null
rm -rf $OUT/ada_trace $OUT/ada_trace0

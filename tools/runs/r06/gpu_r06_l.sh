#!/usr/bin/env bash
# Round 6, session l: the fast pow with one LDS read per table and NaN folded into the exact
# cases (tests, exhaustive check, timing); the f32 logarithm's error over every positive float.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
T="python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu"
run t_ada 600 $T tests/test_adaround_golden.py tests/test_gpu_parity.py -k "adaround"
run pow_check 300 tools/studies/pow_fast_check
run ada_tab 300 python tools/studies/ada_bwd_tune.py --scales 1,4 --tag l_aos
run ada_reg0 300 python tools/studies/ada_bwd_tune.py --scales 1 --reg 0 --tag l_reg0
run ada_tab2 300 python tools/studies/ada_bwd_tune.py --scales 1,4 --tag l_aos_rep
run log_check 300 tools/studies/log_f32_check

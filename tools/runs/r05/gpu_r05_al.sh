#!/usr/bin/env bash
# Round 5, session al: the AdaRound backward without the loss value launched one tile per workgroup
# (library form): the AdaRound GPU tests, the grid-forms test, and the 2^28 tuning runs (reg 0.01, 0).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_adaround_golden.py tests/test_adaround_wrapper.py -k "adaround or ada"
run ada_lib 300 python -u tools/studies/ada_bwd_tune.py --tag lib_full_grid
run ada_lib0 300 python -u tools/studies/ada_bwd_tune.py --reg 0 --tag lib_full_grid_reg0

#!/usr/bin/env bash
# Round 4, session v: the 1x1 / stem one-pass steps' slices folded by the Adam step too -- the AdaRound tests, the
# 2k- and 10k-iteration loops.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_ada 900 python -u -m pytest tests/test_adaround_wrapper.py tests/test_adaround_golden.py tests/test_adaround_dist_gpu.py tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -k "adaround or adam or dw or depthwise or pw_ or pointwise"
run ada2k 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000
AIMET_ADA_DW_FOLD_ADAM=0 run ada2k_fold 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000
run ada10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000

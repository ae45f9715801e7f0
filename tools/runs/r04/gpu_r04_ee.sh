#!/usr/bin/env bash
# Round 4, session ee: the projecting 1x1 layers at 28 x 28 with C_in >= 32 as the one-pass step
# (the shape rule after session dd) -- the AdaRound tests and config 3 at 10k iterations.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_ada 900 python -u -m pytest tests/test_adaround_wrapper.py tests/test_adaround_golden.py tests/test_adaround_dist_gpu.py tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -k "adaround or adam or dw or depthwise or pw_ or pointwise"
run ada10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000

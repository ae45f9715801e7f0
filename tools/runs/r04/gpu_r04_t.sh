#!/usr/bin/env bash
# Round 4, session t: learned-grid tiles back to two groups per lane (lm_head bound); AdaRound
# graphs of 10 vs 50 iterations; the bench line after the calibration host trims.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_lg 900 python -u -m pytest tests/test_gpu_parity.py tests/test_llama_quantsim_gpu.py tests/test_range_learning.py -v --timeout 300 --timeout-method thread -k "learned_grid or lg_ or llama or range"
run ada_tune 300 python -u tools/studies/ada_bwd_tune.py
AIMET_ADA_BWD_OCC=8 run ada_tune_occ8 300 python -u tools/studies/ada_bwd_tune.py
run ada2k 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000
AIMET_ADA_GRAPH_ITERS=50 run ada2k_k50 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000
run bench 600 python -u bench.py

#!/usr/bin/env bash
# Round 6, session e: the AdaRound backward on the f64 pow (tests in both pow forms, 2^28 timing and
# VALU counts beside the exact form), the rewritten entropy search and the pinned MSE / entropy
# results (tests + timing).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
T="python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu"
run t_ada 900 $T tests/test_adaround_golden.py tests/test_gpu_parity.py -k "adaround"
run t_ent 900 $T tests/test_entropy.py tests/test_search_resnet_gpu.py tests/test_gpu_parity.py -k "entropy or search or mse or calibrate or get_encodings"
run ada_f64 300 python tools/studies/ada_bwd_tune.py --scales 1,4 --tag r06_f64
run ada_exact 300 python tools/studies/ada_bwd_tune.py --scales 1,4 --tag r06_exact --exact-pow
run ada_reg0 300 python tools/studies/ada_bwd_tune.py --scales 1 --reg 0 --tag r06_reg0
run search_time 300 python tools/studies/tfe_search_time.py MSE ENTROPY
run search_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/search_trace3 -o run -- python3 tools/studies/tfe_search_time.py MSE ENTROPY
run ada_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ada_trace -o run -- python3 tools/studies/ada_bwd_tune.py --scales 1 --tag trace_f64
run ada_pmc 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/ada_pmc -o run -- python3 tools/studies/ada_bwd_tune.py --scales 1 --reps 1 --tag pmc_f64
run t_wrap 900 $T tests/test_adaround_wrapper.py

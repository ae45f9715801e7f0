#!/usr/bin/env bash
# Round 6, session c: config 1 sharded through the sim (the single process on the ranks' forward
# shapes, oracle-checked), the MSE search (zero-mass bins skipped, guarded reciprocal) against the
# oracle, the calibration plan's event-guarded destruction, and the searches' kernel times.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
T="python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu"
run t_sharded 900 $T tests/test_quantsim_sharded_gpu.py
run t_search 900 $T tests/test_search_resnet_gpu.py
run t_parity 900 $T tests/test_gpu_parity.py -k "search or mse or calibrate or plan or resident"
run t_san 300 $T tests/test_sanitize.py
run search_trace 600 rocprofv3 --kernel-trace --stats -d gpurun_out/search_trace -o run -- python tools/studies/tfe_search_time.py MSE ENTROPY TF_ENHANCED

#!/usr/bin/env bash
# Round 6, session au: the MSE search kernels at 6 waves per SIMD (80 VGPRs, a few spills); the edges
# classified over the workgroup by prefix sums: parity, kernel trace, timing.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
T="python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu"
run t_mse 600 $T tests/test_search_resnet_gpu.py tests/test_gpu_parity.py tests/test_quantsim.py -k "mse or MSE or search or independent or compute_encodings"
run tr_au 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mse_au -o run -- python3 tools/studies/tfe_search_time.py MSE
run search_time 300 python tools/studies/tfe_search_time.py MSE ENTROPY TF_ENHANCED

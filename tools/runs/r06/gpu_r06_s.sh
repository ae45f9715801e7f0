#!/usr/bin/env bash
# Round 6, session s: getEncodings' result objects built while the searches run (parity through
# every batched-encoding caller), then the search timing.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
T="python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu"
run t_enc 900 $T tests/test_entropy.py tests/test_search_resnet_gpu.py tests/test_gpu_parity.py tests/test_quantsim.py tests/test_quantsim_sharded_gpu.py
run search_time 300 python tools/studies/tfe_search_time.py MSE ENTROPY TF_ENHANCED

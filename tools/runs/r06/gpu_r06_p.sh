#!/usr/bin/env bash
# Round 6, session p: entropy encodings finished on the device (only flagged channels on the
# host): parity tests, then the search timing with its phases.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
T="python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu"
run t_ent 600 $T tests/test_entropy.py tests/test_search_resnet_gpu.py tests/test_gpu_parity.py -k "entropy or ENTROPY or search"
run search_time 300 python tools/studies/tfe_search_time.py MSE ENTROPY
run t_qs 600 $T tests/test_quantsim.py

#!/usr/bin/env bash
# Round 6, session av: the entropy kernel at 23.6 KB of LDS and 5 waves per SIMD (6 workgroups per
# CU): parity, kernel trace, timing.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
T="python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu"
run t_ent 600 $T tests/test_entropy.py tests/test_search_resnet_gpu.py tests/test_gpu_parity.py -k "entropy or ENTROPY or search or independent"
run tr_av 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ent_av -o run -- python3 tools/studies/tfe_search_time.py ENTROPY
run search_time 300 python tools/studies/tfe_search_time.py ENTROPY MSE

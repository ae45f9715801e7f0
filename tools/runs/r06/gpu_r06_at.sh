#!/usr/bin/env bash
# Round 6, session at: the MSE search kernels at 6 waves per SIMD (study build, 80 VGPRs with a few
# spills) against the library's 5 (96 VGPRs), alternating kernel traces.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
P="rocprofv3 --kernel-trace --output-format csv"
run tr_w5a 300 $P -d gpurun_out/mse_at_w5a -o run -- python3 tools/studies/tfe_search_time.py MSE
run tr_w6a 300 $P -d gpurun_out/mse_at_w6a -o run -- python3 tools/studies/tfe_search_time.py --lib tools/studies/mse_lib/w6/libaimet_amd.so MSE
run tr_w5b 300 $P -d gpurun_out/mse_at_w5b -o run -- python3 tools/studies/tfe_search_time.py MSE
run tr_w6b 300 $P -d gpurun_out/mse_at_w6b -o run -- python3 tools/studies/tfe_search_time.py --lib tools/studies/mse_lib/w6/libaimet_amd.so MSE

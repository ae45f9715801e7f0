#!/usr/bin/env bash
# Round 6, session ap: the MSE search's per-workgroup preamble (PDF load, one-lane mse::setup, bin
# compaction) -- a study build that evaluates no candidate -- against the full kernel (traces).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
P="rocprofv3 --kernel-trace --output-format csv"
run tr_full 300 $P -d gpurun_out/mse_ap_full -o run -- python3 tools/studies/tfe_search_time.py MSE
run tr_nocand 300 $P -d gpurun_out/mse_ap_nocand -o run -- python3 tools/studies/tfe_search_time.py --lib tools/studies/mse_lib/nocand/libaimet_amd.so MSE

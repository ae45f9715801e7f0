#!/usr/bin/env bash
# Round 6, session q: the entropy search kernel with and without the waves-per-EU hint (kernel
# trace of each, twice, alternating).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
P="rocprofv3 --kernel-trace --stats --output-format csv"
run tr_w4a 300 $P -d gpurun_out/ent_trace_w4a -o run -- python3 tools/studies/tfe_search_time.py ENTROPY
run tr_w3a 300 $P -d gpurun_out/ent_trace_w3a -o run -- python3 tools/studies/tfe_search_time.py --lib tools/studies/ent_lib/w3/libaimet_amd.so ENTROPY
run tr_w4b 300 $P -d gpurun_out/ent_trace_w4b -o run -- python3 tools/studies/tfe_search_time.py ENTROPY
run tr_w3b 300 $P -d gpurun_out/ent_trace_w3b -o run -- python3 tools/studies/tfe_search_time.py --lib tools/studies/ent_lib/w3/libaimet_amd.so ENTROPY

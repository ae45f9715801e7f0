#!/usr/bin/env bash
# Round 6, session y: where the entropy kernel's time goes, symmetric vs asymmetric (study builds
# without step 3 / steps 2-3, tools/studies/ent_variants.sh), kernel traces.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
P="rocprofv3 --kernel-trace --output-format csv"
run tr_full 300 $P -d gpurun_out/ent_y_full -o run -- python3 tools/studies/tfe_search_time.py ENTROPY
run tr_no3 300 $P -d gpurun_out/ent_y_no3 -o run -- python3 tools/studies/tfe_search_time.py --lib tools/studies/ent_lib/no3/libaimet_amd.so ENTROPY
run tr_no23 300 $P -d gpurun_out/ent_y_no23 -o run -- python3 tools/studies/tfe_search_time.py --lib tools/studies/ent_lib/no23/libaimet_amd.so ENTROPY

#!/usr/bin/env bash
# Round 6, session ac: the entropy kernel's asymmetric remainder -- study builds without steps 2-3,
# with and without the asymmetric window walk (kernel traces).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
P="rocprofv3 --kernel-trace --output-format csv"
run tr_no23 300 $P -d gpurun_out/ent_ac_no23 -o run -- python3 tools/studies/tfe_search_time.py --lib tools/studies/ent_lib/no23/libaimet_amd.so ENTROPY
run tr_no23w 300 $P -d gpurun_out/ent_ac_no23w -o run -- python3 tools/studies/tfe_search_time.py --lib tools/studies/ent_lib/no23w/libaimet_amd.so ENTROPY

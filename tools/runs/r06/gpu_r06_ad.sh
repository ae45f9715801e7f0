#!/usr/bin/env bash
# Round 6, session ad: the asymmetric window walk -- entropy::windows vs the prefetching walk
# (ent_walk_variant.py), with and without steps 2-3 (kernel traces).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
P="rocprofv3 --kernel-trace --output-format csv"
for v in no23 no23fw no23w fw; do
  run tr_$v 300 $P -d gpurun_out/ent_ad_$v -o run -- python3 tools/studies/tfe_search_time.py --lib tools/studies/ent_lib/$v/libaimet_amd.so ENTROPY
done
run tr_prod 300 $P -d gpurun_out/ent_ad_prod -o run -- python3 tools/studies/tfe_search_time.py ENTROPY

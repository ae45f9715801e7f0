#!/usr/bin/env bash
# Round 5, session m: AdaRound backward occupancy (launch bounds for 6/7/8 waves per SIMD) x grid size
# (8192 = 5.3 rounds of resident workgroups, or exactly 1 or 2 rounds) at 2^28 elements. Ran against
# temporary builds (launch bounds -DADA_BWD_WAVES=W, grid cap read from AIMET_TMP_ADA_GRID) that were
# removed after the sweep: every form within noise of the library's (profiles/r05/ada_bwd_occ_grid.jsonl).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
for W in 6 7 8; do
  for G in 8192 $((256 * W)) $((512 * W)); do
    AIMET_TMP_ADA_GRID=$G run ada_w${W}_g$G 120 python -u tools/studies/ada_bwd_tune.py --lib tools/studies/exp_libs/lib_w$W.so --tag w${W}_g$G
    grep -h '^{' $OUT/ada_w${W}_g$G.log >> $OUT/ada_occ_grid.jsonl
  done
done

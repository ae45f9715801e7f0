#!/usr/bin/env bash
# Round 5, session u: where the parameters' calibration work runs beside the activations' passes --
# temporary builds (removed after): the parameters' TF-E search capped at 1 / 2 / 4 workgroups per
# CU beside the min/max pass; the search (late1) or the statistics and the search (late2) queued
# after the min/max pass, i.e. beside the histogram pass. tools/studies/enc_plan_runs.py, form both.
# Result (profiles/r05/enc_sched_variants.jsonl): the library's form (2 per CU, beside the min/max
# pass) 3.65-3.68 ms; 1 per CU 5.48 (the host waits for the parameters' encodings), 4 per CU 3.76,
# late1 4.63 (capped) / 3.91 (uncapped), late2 4.69.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
for L in pcu2 pcu1 pcu4 late1_pcu2 late1_pcu0 late2_pcu2 pcu2; do
  run enc_$L 240 python -u tools/studies/enc_plan_runs.py --reps 30 --forms both --lib tools/studies/exp_libs/lib_$L.so --tag $L
  grep -h '^{' $OUT/enc_$L.log >> $OUT/enc_sched_variants.jsonl
done

#!/usr/bin/env bash
# Round 5, session as: the AdaRound backward per element at sizes whose 4 buffers stay in the
# Infinity Cache (2^20, 2^22 elements: 16 / 64 MB) against 2^24 and 2^28 -- is the pow form's time
# the arithmetic alone, or arithmetic and memory not overlapped?
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
for E in 20 22 24 28; do
  run ada_size_$E 300 python -u tools/studies/ada_bwd_tune.py --scales 1 --elems $((1 << E)) --channels 64 --reps 50 --tag size_2e$E
  run ada_size0_$E 300 python -u tools/studies/ada_bwd_tune.py --scales 1 --elems $((1 << E)) --channels 64 --reps 50 --reg 0 --tag size_2e${E}_reg0
done
grep -h '^{' $OUT/ada_size_*.log $OUT/ada_size0_*.log > $OUT/ada_bwd_sizes.jsonl

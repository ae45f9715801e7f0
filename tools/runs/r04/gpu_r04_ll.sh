#!/usr/bin/env bash
# Round 4, session ll: five bench lines at the final tree in one process each (the spread of the
# value and of compute_encodings' fraction run to run).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
for i in 1 2 3 4 5; do
  run bench_rep$i 300 python -u bench.py --no-cpu-baseline
done

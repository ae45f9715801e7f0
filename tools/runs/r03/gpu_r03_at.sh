#!/usr/bin/env bash
# Round 3: compute_encodings as two native calls (activations first, the parameters' host
# preparation beside their min/max pass) vs one call (AIMET_CAL_SPLIT=0); whole GPU suite, smoke, bench.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
grep -q " passed" $OUT/gpu_tests.log && ! grep -q " failed\| error" $OUT/gpu_tests.log || { echo "tests failed"; exit 1; }
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
for i in 1 2; do
  run bench_split_$i 300 python -u bench.py
  AIMET_CAL_SPLIT=0 run bench_one_$i 300 python -u bench.py --steps 20
done
grep -o '"compute_encodings_s": [0-9.]*\|"frac": 0.7[0-9]*' $OUT/bench_*.log

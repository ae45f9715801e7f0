#!/usr/bin/env bash
# Round 3: request discard on the two-call error path; the whole GPU suite, smoke, bench.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
grep -q " passed" $OUT/gpu_tests.log && ! grep -q " failed\| error" $OUT/gpu_tests.log || { echo "tests failed"; exit 1; }
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 300 python -u bench.py

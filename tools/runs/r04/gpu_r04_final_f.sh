#!/usr/bin/env bash
# Round 4 closing check F (final tree: the measured CPU compute_encodings baseline, the 28 x 28
# projecting-layer rule, the config-5 first-step dump): the whole GPU suite, smoke, the default
# bench line.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run gpu_tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 900 python -u bench.py

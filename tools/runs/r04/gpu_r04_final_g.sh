#!/usr/bin/env bash
# Round 4 closing check G (final tree): the whole GPU suite and smoke.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run gpu_tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"

#!/usr/bin/env bash
# Round 5, session n: checkpoint of the tree after the AdaRound packed-pow change -- the whole GPU
# suite and smoke().
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run gpu_tests 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')"

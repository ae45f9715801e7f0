#!/usr/bin/env bash
# Round 6, closing check T (1/2): the whole GPU suite, smoke(), and the default bench line
# (headline + drop-in + configs 3 and 5).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run gpu_suite 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 720 python bench.py

#!/usr/bin/env bash
# Round 5, closing check T (run again as T2 after the drop-in changes): the whole GPU suite and smoke() at
# the tree, then the default bench line
# twice and the --force-exchange line.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run gpu_tests 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')"
run bench1 600 python -u bench.py
run bench2 400 python -u bench.py --no-cpu-baseline --no-dropin
run bench_x 400 python -u bench.py --no-cpu-baseline --no-dropin --force-exchange

#!/usr/bin/env bash
# end-of-round check: smoke, every GPU test, the bench line
source "$(dirname "$0")/gpu_lib.sh"
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 1200 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests
run bench 600 python bench.py
echo ALLDONE

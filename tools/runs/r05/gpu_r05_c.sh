#!/usr/bin/env bash
# Round 5, session c: the whole GPU suite after the calibration-plan refactor and the removal of the
# tuning switches, then the plan timing forms (incl. bench.py's preamble) and the default bench line.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run gpu_tests 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
run enc_runs 300 python -u tools/studies/enc_plan_runs.py --reps 30
run bench 400 python -u bench.py --force-exchange

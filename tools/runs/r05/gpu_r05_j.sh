#!/usr/bin/env bash
# Round 5, session j: the default bench line after the harness fix (previous results released
# before the clock), twice, and the force-exchange line.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run bench1 600 python -u bench.py
run bench2 400 python -u bench.py --no-cpu-baseline --force-exchange

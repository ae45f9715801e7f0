#!/usr/bin/env bash
# Round 5, session d: bench.py with per-run GPU spans of the plan (sim's quantizers vs a new sim).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run bench 400 python -u bench.py --no-cpu-baseline --no-dropin

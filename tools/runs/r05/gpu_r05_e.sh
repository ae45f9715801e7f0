#!/usr/bin/env bash
# Round 5, session e: host phases of the plan's compute_encodings in bench.py vs the study process.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run enc_runs 300 python -u tools/studies/enc_plan_runs.py --reps 20
run bench 400 python -u bench.py --no-cpu-baseline --no-dropin

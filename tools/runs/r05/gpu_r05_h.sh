#!/usr/bin/env bash
# Round 5, session h: the parameters' search held to 2 workgroups per CU beside the min/max pass;
# request events polled; plan forms and the bench line.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_cal 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "calib or encoding or resident or bench_calibration or plan"
run enc_runs 300 python -u tools/studies/enc_plan_runs.py --reps 20 --forms both,acts,both_after_resident
run bench 400 python -u bench.py --no-cpu-baseline --no-dropin

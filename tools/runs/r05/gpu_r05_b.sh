#!/usr/bin/env bash
# Round 5, session b: where the plan's compute_encodings time goes (per-run wall vs GPU span, the
# parts alone), the default bench line (drop-in surface fields), the full-shape Llama tests.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run enc_runs 300 python -u tools/studies/enc_plan_runs.py --reps 30
run bench 400 python -u bench.py --force-exchange
run t_llama 900 python -u -m pytest tests/test_llama_quantsim_gpu.py -v --timeout 600 --timeout-method thread

#!/usr/bin/env bash
# Round 5, session z2: the ANALYSIS forwards' activation statistics batched per forward (StatsBatch)
# -- the quantsim / config-1 oracle / DataParallel / checkpoint / range-learning tests, the drop-in
# profile and a bench line with the drop-in fields.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_q 900 python -u -m pytest tests/test_quantsim.py tests/test_range_learning.py tests/test_checkpoint.py tests/test_dropin_boundary.py tests/test_configs_gpu.py tests/test_llama_quantsim_gpu.py tests/test_qat_ddp_gpu.py -q --timeout 600 --timeout-method thread -m gpu -k "not config4"
run dropin_prof 300 python -u tools/studies/dropin_profile.py --reps 3
run bench 400 python -u bench.py --no-cpu-baseline

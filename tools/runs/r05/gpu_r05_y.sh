#!/usr/bin/env bash
# Round 5, session y: QuantizationSimModel.compute_encodings with the parameter encodings computed up
# front in batched calls -- the quantsim / config-1 / checkpoint / range-learning / DataParallel tests
# and the drop-in profile.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_qs 900 python -u -m pytest tests/test_quantsim.py tests/test_configs_gpu.py tests/test_checkpoint.py tests/test_range_learning.py tests/test_dropin_boundary.py tests/test_qat_ddp_gpu.py tests/test_llama_quantsim_gpu.py -v --timeout 600 --timeout-method thread -m gpu -k "not config4"
run dropin_prof 300 python -u tools/studies/dropin_profile.py --reps 3

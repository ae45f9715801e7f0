#!/usr/bin/env bash
# Round 5, session ac: StatsBatch copies the tensors it queues (in-place ops after a quantized output:
# nn.ReLU(inplace=True), `out += identity`) -- quantsim / config-1 / DataParallel tests, drop-in profile.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_q 900 python -u -m pytest tests/test_quantsim.py tests/test_dropin_boundary.py tests/test_configs_gpu.py tests/test_range_learning.py tests/test_checkpoint.py -q --timeout 600 --timeout-method thread -m gpu -k "not config4"
run dropin_prof 300 python -u tools/studies/dropin_profile.py --reps 3

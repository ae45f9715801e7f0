#!/usr/bin/env bash
# Round 5, session z: StaticGridTensorQuantizer.quantize_dequantize without the autograd call when
# no graph would be recorded -- the suites that QDQ through the quantizers, the drop-in profile and
# a bench line with the drop-in fields.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_q 900 python -u -m pytest tests/test_quantsim.py tests/test_range_learning.py tests/test_checkpoint.py tests/test_dropin_boundary.py tests/test_adaround_wrapper.py tests/test_configs_gpu.py tests/test_gpu_parity.py -q --timeout 600 --timeout-method thread -m gpu -k "not config4"
run dropin_prof 300 python -u tools/studies/dropin_profile.py --reps 3
run bench 400 python -u bench.py --no-cpu-baseline

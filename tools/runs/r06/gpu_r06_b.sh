#!/usr/bin/env bash
# Round 6, session b: sharded calibration through the drop-in QuantizationSimModel (config 1 split
# 16 + 16, the in-place / copy tests, config 4 through the sim, config 5's DDP worker on shards),
# the quantsim regression tests, and the drop-in profile after the StatsBatch / parameter-cache change.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
T="python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu"
run t_sharded 900 $T tests/test_quantsim_sharded_gpu.py
run t_qs 600 $T tests/test_quantsim.py tests/test_dropin_boundary.py tests/test_checkpoint.py
run t_ddp 600 $T tests/test_qat_ddp_gpu.py
run dropin 300 python tools/studies/dropin_profile.py --reps 3
run t_cfg 1200 $T tests/test_configs_gpu.py

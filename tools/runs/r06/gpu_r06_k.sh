#!/usr/bin/env bash
# Round 6, session k: config 5 after bounding the calibration's parameter-QDQ cache (this tree vs
# the round-5 tree); the quantsim tests; the drop-in phases; where the AdaRound fast pow's time
# goes (study builds without its LDS table reads / without the table barrier).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
T="python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu"
run llama_r06 600 python -u benchmarks/llama_qat.py --steps 5 --warmup 2
run llama_r05 600 python -u tools/studies/r05tree/benchmarks/llama_qat.py --steps 5 --warmup 2
run llama_r06b 600 python -u benchmarks/llama_qat.py --steps 5 --warmup 2
run t_qs 900 $T tests/test_quantsim.py tests/test_quantsim_sharded_gpu.py
run dropin 300 python tools/studies/dropin_profile.py
run ada_base 300 python tools/studies/ada_bwd_tune.py --scales 1 --tag k_base
run ada_nolds 300 python tools/studies/ada_bwd_tune.py --scales 1 --tag k_nolds --lib tools/studies/ada_lib/nolds/libaimet_amd.so
run ada_nobar 300 python tools/studies/ada_bwd_tune.py --scales 1 --tag k_nobar --lib tools/studies/ada_lib/nobar/libaimet_amd.so
run ada_base2 300 python tools/studies/ada_bwd_tune.py --scales 1 --tag k_base2

#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_lg 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_range_learning.py tests/test_configs_gpu.py -k "learned or range or lg or qat or config5 or golden"
run llama 600 python -u benchmarks/llama_qat.py --path quantsim --layers 32 --steps 5 --warmup 2
run llama2 600 python -u benchmarks/llama_qat.py --path quantsim --layers 32 --steps 5 --warmup 2
echo ALLDONE

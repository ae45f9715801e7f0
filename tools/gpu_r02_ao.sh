#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_lg 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_range_learning.py tests/test_configs_gpu.py tests/test_distributed_gpu.py -k "learned or range or lg or qat or config or many or minmax or hist or shard"
run llama 600 python -u benchmarks/llama_qat.py --path quantsim --layers 32 --steps 5 --warmup 2
run vit 300 python -u benchmarks/vit_calibration.py
run tune 400 python -u tools/enc_partition_tune.py params_first:0 params_first:0
echo ALLDONE

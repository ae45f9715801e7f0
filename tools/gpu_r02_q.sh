#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run lg16 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py -k "learned_grid"
run llama 600 python -u benchmarks/llama_qat.py --path quantsim --layers 32 --steps 5 --warmup 2
run resnet_cpu 600 python -u benchmarks/resnet_quantsim.py --cpu-model
echo ALLDONE

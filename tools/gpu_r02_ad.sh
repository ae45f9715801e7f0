#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run llama_ref 600 python -u benchmarks/llama_qat.py --path quantsim --impl reference --layers 32 --steps 5 --warmup 2
run llama 600 python -u benchmarks/llama_qat.py --path quantsim --layers 32 --steps 5 --warmup 2
run rq_cpu 900 python -u benchmarks/resnet_quantsim.py --cpu-model --repeats 3
echo ALLDONE

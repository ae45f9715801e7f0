#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run rq_gpu 600 python -u benchmarks/resnet_quantsim.py --repeats 3
run rq_cpu 900 python -u benchmarks/resnet_quantsim.py --cpu-model --repeats 3
echo ALLDONE

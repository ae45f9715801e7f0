#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run ada_warm 300 python -u benchmarks/adaround_mobilenet.py --iterations 300
run ada_10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000 --reference-iters 300
echo ALLDONE

#!/usr/bin/env bash
# Round 5, session s: the N-rank bench path rehearsed with 2 ranks on the one GPU over gloo (the
# calibration plan's staged launch with its collectives), then configs 3, 4 and 5 re-measured at
# this tree.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
AIMET_BENCH_BACKEND=gloo run bench_gloo2 400 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --no-dropin --enc-reps 2 --plan-reps 5
run ada10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000
run vit 600 python -u benchmarks/vit_calibration.py --images 160
run llama 900 python -u benchmarks/llama_qat.py --steps 5 --warmup 2

#!/usr/bin/env bash
# Round 5, session ab: the N-rank bench path rehearsed with 4 ranks on the one GPU over gloo.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
AIMET_BENCH_BACKEND=gloo run bench_gloo4 600 python -u bench.py --gpus 4 --steps 10 --warmup 2 --no-cpu-baseline --no-dropin --enc-reps 2 --plan-reps 5

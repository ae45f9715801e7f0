#!/usr/bin/env bash
# Round 6, session ao: the N-rank bench path at the final tree, rehearsed with 2 and 4 ranks on the
# one GPU over gloo (the driver runs N = 1, 2, 4, 8 over RCCL on an 8-GPU node), plus the
# multi-rank GPU tests (sharded QuantizationSimModel calibration, RCCL world-1 exchange).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
AIMET_BENCH_BACKEND=gloo run bench_gloo2 400 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --no-dropin --enc-reps 2 --plan-reps 5 --no-secondary
AIMET_BENCH_BACKEND=gloo run bench_gloo4 600 python -u bench.py --gpus 4 --steps 10 --warmup 2 --no-cpu-baseline --no-dropin --enc-reps 2 --plan-reps 5 --no-secondary

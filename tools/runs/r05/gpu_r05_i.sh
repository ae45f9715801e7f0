#!/usr/bin/env bash
# Round 5, session i: bench.py's host gap after the GPU span (enc_bench_host variants).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run enc_host 300 python -u tools/studies/enc_bench_host.py --reps 20

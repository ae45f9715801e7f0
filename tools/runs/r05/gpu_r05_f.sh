#!/usr/bin/env bash
# Round 5, session f: host split of bench.py's plan runs (tools/studies/enc_bench_host.py).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run enc_host 300 python -u tools/studies/enc_bench_host.py --reps 20

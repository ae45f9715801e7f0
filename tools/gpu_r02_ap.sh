#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run llama 600 python -u benchmarks/llama_qat.py --path quantsim --layers 32 --steps 5 --warmup 2
run llama_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/lp" -o run -- python3 benchmarks/llama_qat.py --path quantsim --layers 32 --steps 3 --warmup 1
rm -f "$OUT"/lp/*kernel_trace.csv
run llama2 600 python -u benchmarks/llama_qat.py --path quantsim --layers 32 --steps 5 --warmup 2
echo ALLDONE

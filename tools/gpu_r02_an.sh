#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run llama_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/lp" -o run -- python3 benchmarks/llama_qat.py --path quantsim --layers 32 --steps 3 --warmup 1
rm -f "$OUT"/lp/*kernel_trace.csv
run vit 300 python -u benchmarks/vit_calibration.py
run vit2 300 python -u benchmarks/vit_calibration.py --oracle-check 0
echo ALLDONE

#!/usr/bin/env bash
# kernel time of the Llama-3-8B QuantSim QAT step (stats only; the per-dispatch trace is deleted)
source "$(dirname "$0")/gpu_lib.sh"
run llama_prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/llama_prof" -o run --output-format csv -- python3 -u benchmarks/llama_qat.py --path quantsim --layers 32 --steps 3 --warmup 1
rm -f "$OUT"/llama_prof/*kernel_trace.csv
echo ALLDONE

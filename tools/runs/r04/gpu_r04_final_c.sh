#!/usr/bin/env bash
# Round 4 closing check C: config 3 (AdaRound 10k) and the trace of the adopted loop, config 5 (Llama
# QAT step through QuantizationSimModel), config 4 (ViT-L/16 calibration, oracle-checked batch).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000
run ada_trace 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/ada_trace -o run -- python3 benchmarks/adaround_mobilenet.py --iterations 200
python tools/studies/ada_trace_summary.py $OUT/ada_trace $((53*200)) > $OUT/ada_trace_summary.txt 2>&1
rm -rf $OUT/ada_trace
run llama 600 python -u benchmarks/llama_qat.py --steps 5 --warmup 2
run vit 600 python -u benchmarks/vit_calibration.py --images 160
AIMET_ADA_BWD_OCC=8 run ada_tune_occ8 300 python -u tools/studies/ada_bwd_tune.py

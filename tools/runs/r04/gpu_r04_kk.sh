#!/usr/bin/env bash
# Round 4, session kk: configs 4 and 5 at the final tree (ViT-L/16 calibration with every batch's
# encodings checked against the CPU oracle; the Llama-3-8B QAT step through QuantizationSimModel).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run vit 600 python -u benchmarks/vit_calibration.py --images 160
run llama 600 python -u benchmarks/llama_qat.py --steps 5 --warmup 2

#!/usr/bin/env bash
# Round 4, session cc: config 5 at full size, first step parity -- Llama-3-8B W4A16 learned-grid QAT
# through QuantizationSimModel with our kernels and with the reference's torch-op
# QuantizeDequantize, same seeds: loss and weight-gradient sums bit for bit, range gradients'
# relative error (tools/studies/llama_first_step_compare.py).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run llama_first_fused 600 python -u benchmarks/llama_qat.py --steps 1 --warmup 0 --impl fused --dump-first $OUT/llama_first_fused.pt
run llama_first_ref 600 python -u benchmarks/llama_qat.py --steps 1 --warmup 0 --impl reference --dump-first $OUT/llama_first_ref.pt
python tools/studies/llama_first_step_compare.py $OUT/llama_first_fused.pt $OUT/llama_first_ref.pt > $OUT/llama_first_step_compare.json 2>&1
rm -f $OUT/llama_first_fused.pt $OUT/llama_first_ref.pt

#!/usr/bin/env bash
# Round 3: 16-bit learned-grid kernels with / without nontemporal accesses; Llama-3-8B QAT step.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run lg16_tests 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "learned_grid and (16 or non_finite)"
for nt in 1 0 1 0; do
  i=$((i+1))
  run lgn$i 200 env AIMET_TUNE_LG16_NT=$nt rocprofv3 --kernel-trace --output-format csv -d $OUT/lgn$i -o run -- python3 benchmarks/lg16_roofline.py --reps 40
  python3 tools/studies/lg16_trace_summary.py $OUT/lgn$i "nt=$nt" >> $OUT/lg_nt.jsonl
done
run llama_nt1 600 python -u benchmarks/llama_qat.py --steps 5 --warmup 2
run llama_nt0 600 env AIMET_TUNE_LG16_NT=0 python -u benchmarks/llama_qat.py --steps 5 --warmup 2

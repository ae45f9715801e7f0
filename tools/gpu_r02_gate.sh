#!/usr/bin/env bash
# a wrapper's range gates in one launch: parity, then the QAT step and its kernel profile
source "$(dirname "$0")/gpu_lib.sh"
run t_gate 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_range_learning.py tests/test_configs_gpu.py -k "learned or range or lg or qat or config5 or golden or gate"
grep -q " passed" "$OUT/t_gate.log" && ! grep -q "failed" "$OUT/t_gate.log" || { echo "tests failed"; exit 1; }
run llama_g1 600 python -u benchmarks/llama_qat.py --path quantsim --layers 32 --steps 5 --warmup 2
run llama_g2 600 python -u benchmarks/llama_qat.py --path quantsim --layers 32 --steps 5 --warmup 2
run llama_prof_gate 600 rocprofv3 --kernel-trace --stats -d "$OUT/llama_prof_gate" -o run --output-format csv -- python3 -u benchmarks/llama_qat.py --path quantsim --layers 32 --steps 3 --warmup 1
rm -f "$OUT"/llama_prof_gate/*kernel_trace.csv
echo ALLDONE

#!/usr/bin/env bash
# learned-grid forward: two quads per lane (default) vs one (AIMET_TUNE_LG_FWD_QUADS=1), A/B/A
source "$(dirname "$0")/gpu_lib.sh"
run t_lg 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_range_learning.py tests/test_configs_gpu.py -k "learned or range or lg or qat or config5 or golden"
grep -q " passed" "$OUT/t_lg.log" && ! grep -q "failed" "$OUT/t_lg.log" || { echo "tests failed"; exit 1; }
run llama_q2a 600 python -u benchmarks/llama_qat.py --path quantsim --layers 32 --steps 5 --warmup 2
AIMET_TUNE_LG_FWD_QUADS=1 run llama_q1 600 python -u benchmarks/llama_qat.py --path quantsim --layers 32 --steps 5 --warmup 2
run llama_q2b 600 python -u benchmarks/llama_qat.py --path quantsim --layers 32 --steps 5 --warmup 2
run llama_prof2 600 rocprofv3 --kernel-trace --stats -d "$OUT/llama_prof2" -o run --output-format csv -- python3 -u benchmarks/llama_qat.py --path quantsim --layers 32 --steps 3 --warmup 1
rm -f "$OUT"/llama_prof2/*kernel_trace.csv
echo ALLDONE

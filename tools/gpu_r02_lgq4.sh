#!/usr/bin/env bash
# learned-grid forward kernel time: four quads per lane vs two (rocprofv3 stats of the QAT step)
source "$(dirname "$0")/gpu_lib.sh"
AIMET_TUNE_LG_FWD_QUADS=4 run t_lg4 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_range_learning.py -k "learned or range or lg"
grep -q " passed" "$OUT/t_lg4.log" && ! grep -q "failed" "$OUT/t_lg4.log" || { echo "tests failed"; exit 1; }
for q in 4 2; do
  AIMET_TUNE_LG_FWD_QUADS=$q run llama_prof_q$q 600 rocprofv3 --kernel-trace --stats -d "$OUT/llama_prof_q$q" -o run --output-format csv -- python3 -u benchmarks/llama_qat.py --path quantsim --layers 32 --steps 3 --warmup 1
  rm -f "$OUT"/llama_prof_q$q/*kernel_trace.csv
done
echo ALLDONE

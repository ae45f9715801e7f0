#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
export AIMET_TUNE_MINMAX_TILE=1
run t_many 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_configs_gpu.py tests/test_distributed_gpu.py -k "many or bench or sharded or config1"
run bench_tile 300 python bench.py --no-cpu-baseline
run prof_tile 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_tile" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
export AIMET_TUNE_MINMAX_TILE=0
run bench_grid 300 python bench.py --no-cpu-baseline
rm -f "$OUT"/prof_tile/*kernel_trace.csv
echo ALLDONE

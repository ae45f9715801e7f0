#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_st 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_configs_gpu.py tests/test_distributed_gpu.py -k "hist or many or entropy or tf_ or golden or config or calibrate or resident or percentile or mse or shard"
run pk 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pk" -o run -- python3 tools/pass_kernel_times.py acts
rm -f "$OUT"/pk/*kernel_trace.csv
run vit 600 python -u benchmarks/vit_calibration.py
run bench 300 python bench.py
echo ALLDONE

#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_st 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_configs_gpu.py -k "minmax or many or hist or entropy or tf_ or golden or config1 or calibrate or resident"
run pk 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pk" -o run -- python3 tools/pass_kernel_times.py
rm -f "$OUT"/pk/*kernel_trace.csv
run split 300 python -u tools/enc_split_time.py
echo ALLDONE

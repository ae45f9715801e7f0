#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_tfe 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_configs_gpu.py -k "tfe or search or config or calibrate or resident or golden or channel or many"
run pk 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pk" -o run -- python3 tools/pass_kernel_times.py acts
rm -f "$OUT"/pk/*kernel_trace.csv
run tune 400 python -u tools/enc_partition_tune.py params_first:0 params_first:0
echo ALLDONE

#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run pkw 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pkw" -o run -- python3 tools/pass_kernel_times.py weights
rm -f "$OUT"/pkw/*kernel_trace.csv
run t_tfe 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py -k "tfe or search"
echo ALLDONE

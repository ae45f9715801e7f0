#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_st 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py -k "many or minmax"
run pk 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pk" -o run -- python3 tools/pass_kernel_times.py acts
rm -f "$OUT"/pk/*kernel_trace.csv
run vit 300 python -u benchmarks/vit_calibration.py --oracle-check 0
echo ALLDONE

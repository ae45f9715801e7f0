#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_many 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_configs_gpu.py -k "many or calibrate or resident or config1 or channel"
run split 300 python -u tools/enc_split_time.py
run split_trace 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/split_tr" -o run -- python3 tools/enc_split_time.py
run tl 60 python tools/trace_timeline.py "$OUT/split_tr/run_kernel_trace.csv" minmax_many_kernel 10 14
rm -f "$OUT"/split_tr/*kernel_trace.csv
echo ALLDONE

#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_mm 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py -k "minmax or many or tf_"
run ceil 300 python -u tools/read_ceiling.py
run split 300 python -u tools/enc_split_time.py
echo ALLDONE

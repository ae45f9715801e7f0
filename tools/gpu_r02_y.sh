#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run tune 800 python -u tools/enc_partition_tune.py params_first:0:0:65536 params_first:0:0:256 params_first:0:0:512 params_first:0:0:1024 params_first:0:0:128 params_first:0:0:2048 params_first:0:0:65536
echo ALLDONE

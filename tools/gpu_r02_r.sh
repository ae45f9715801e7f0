#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run probe 120 python -u tools/cu_mask_probe.py
run tune 900 python -u tools/enc_partition_tune.py
echo ALLDONE

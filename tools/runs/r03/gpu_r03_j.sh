#!/usr/bin/env bash
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run vitprof 300 python -u benchmarks/vit_calibration.py --images 96 --oracle-check 0 --profile-host

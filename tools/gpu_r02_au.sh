#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
export AIMET_ADA_DW_ROWS=1
run ada_rows1 600 python -u benchmarks/adaround_mobilenet.py --iterations 3000
export AIMET_ADA_DW_ROWS=0
run ada_gather 600 python -u benchmarks/adaround_mobilenet.py --iterations 3000
export AIMET_ADA_DW_ROWS=1
run ada_rows2 600 python -u benchmarks/adaround_mobilenet.py --iterations 3000
echo ALLDONE

#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run vit_def 300 python -u benchmarks/vit_calibration.py --oracle-check 0
export AIMET_TUNE_HIST_ELEMS=524288; run vit_512k 300 python -u benchmarks/vit_calibration.py --oracle-check 0
export AIMET_TUNE_HIST_ELEMS=32768; run vit_32k 300 python -u benchmarks/vit_calibration.py --oracle-check 0
unset AIMET_TUNE_HIST_ELEMS; export AIMET_TUNE_HIST_BLOCK=1024; run vit_b1024 300 python -u benchmarks/vit_calibration.py --oracle-check 0
export AIMET_TUNE_HIST_BLOCK=256; run vit_b256 300 python -u benchmarks/vit_calibration.py --oracle-check 0
echo ALLDONE

#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
export AIMET_ADA_FUSE_WQ=1
run ada_fuse1 600 python -u benchmarks/adaround_mobilenet.py --iterations 3000
export AIMET_ADA_FUSE_WQ=0
run ada_nofuse 600 python -u benchmarks/adaround_mobilenet.py --iterations 3000
export AIMET_ADA_FUSE_WQ=1
run ada_fuse2 600 python -u benchmarks/adaround_mobilenet.py --iterations 3000
echo ALLDONE

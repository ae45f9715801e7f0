#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
for mu in 2 4 8; do
  AIMET_TUNE_MINMAX_U=$mu AIMET_TUNE_HIST_U=$mu run tune_u$mu 200 python tools/read_ceiling.py
done
AIMET_TUNE_HIST_ELEMS=262144 run tune_e256k 200 python tools/read_ceiling.py
AIMET_TUNE_HIST_ELEMS=65536 run tune_e64k 200 python tools/read_ceiling.py
AIMET_TUNE_HIST_BLOCK=256 AIMET_TUNE_HIST_U=8 run tune_b256u8 200 python tools/read_ceiling.py
echo ALLDONE

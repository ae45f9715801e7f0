#!/usr/bin/env bash
# Round 3: AdaRound pointwise weight-gradient forms (bmm + sum / addbmm / one mm).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
for f in bmm addbmm mm; do
  run ada_$f 600 env AIMET_ADA_PW_GRAD=$f python -u benchmarks/adaround_mobilenet.py --iterations 2000
done

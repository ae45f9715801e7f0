#!/usr/bin/env bash
# Round 3: AdaRound im2col stem form; per-layer form timing under deterministic MIOpen.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "adaround"
run ada_gemm 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000
run ada_timed 600 env AIMET_ADA_LOOP_FORM=timed python -u benchmarks/adaround_mobilenet.py --iterations 2000

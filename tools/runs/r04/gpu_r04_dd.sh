#!/usr/bin/env bash
# Round 4, session dd: which 1x1 layers run faster as the one-pass step now that it uses the matrix
# cores for C_in >= 32 -- the 2k-iteration loop with every eligible layer fused (AIMET_ADA_PW_FUSED=all)
# against the default shape rule, per-layer times compared.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada2k_default 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000
AIMET_ADA_PW_FUSED=all run ada2k_all 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000

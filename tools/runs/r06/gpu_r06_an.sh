#!/usr/bin/env bash
# Round 6, session an: getEncodings' result objects independent across calls (all four searched
# schemes).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_enc 600 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "independent"

#!/usr/bin/env bash
# Round 5, session z4: the batched compute_encodings forms against the per-call forms (quantsim tests).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_qs 600 python -u -m pytest tests/test_quantsim.py tests/test_dropin_boundary.py -v --timeout 600 --timeout-method thread -m gpu

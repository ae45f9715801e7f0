#!/usr/bin/env bash
# Round 5, session q: new GPU tests -- dense (packed) vs compacted rounding-loss pows bit for bit,
# and the fused AdaRound loop's decisions against the reference's torch-op loop.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_new 900 python -u -m pytest tests/test_gpu_parity.py tests/test_adaround_wrapper.py tests/test_adaround_golden.py -v --timeout 300 --timeout-method thread -k "dense_waves or loop_decisions or golden or round_loss"

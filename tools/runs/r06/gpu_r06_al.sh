#!/usr/bin/env bash
# Round 6, session al: AdaRound special values (NaN, inf, the sigmoid's range clamps, tiny negative
# weights) against torch's CPU ops, with the golden tests.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_ada 600 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_adaround_golden.py

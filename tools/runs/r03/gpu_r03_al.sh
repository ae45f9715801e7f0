#!/usr/bin/env bash
# Round 3: learned-grid encoding gradients held to a stated sum bound (float64 reference); the
# AdaRound loop's hard rounding identical wherever alpha is outside the alpha tolerance.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run lg_bound 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "learned_grid_vs_reference_golden or learned_grid_large_vs_torch_ref or matches_reference_loop"

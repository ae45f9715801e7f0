#!/usr/bin/env bash
# Round 6, session am: the rounding-loss gradient's sign by copysign where reg, beta, beta - 1 > 0 (product)
# against HEAD's kernel (study build), alternating; parity and the wrapper loop tests first.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
T="python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu"
run t_ada 600 $T tests/test_adaround_golden.py tests/test_gpu_parity.py tests/test_adaround_wrapper.py -k "adaround or loop or special"
B=tools/studies/ada_lib/base/libaimet_amd.so
for r in 1 2 3; do
  run new$r 300 python tools/studies/ada_bwd_tune.py --scales 1,4 --tag new
  run base$r 300 python tools/studies/ada_bwd_tune.py --scales 1,4 --tag base --lib $B
done

#!/usr/bin/env bash
# Round 4, session m: Adam bias corrections from a per-step table; channel-major gather /
# reconstruction gradient flat with 16-B lanes -- parity, then the 2k-iteration loop.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_ada 900 python -u -m pytest tests/test_adaround_wrapper.py tests/test_adaround_golden.py tests/test_adaround_dist_gpu.py -v --timeout 300 --timeout-method thread
run t_parity 900 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "adaround or adam or pw_cm or learned_grid or lg_"
run ada2k 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000
run pw_cm 300 python -u tools/studies/pw_cm_bench.py --reps 100 --forms library

#!/usr/bin/env bash
# Round 4, session r: channel-major MFMA forward v4 (32-position tiles, prefetched epilogue operands)
# and the wgrad loader for 7x7; the AdaRound backward specialised on the loss value.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_cm 600 python -u -m pytest tests/test_gpu_parity.py tests/test_adaround_wrapper.py tests/test_adaround_golden.py -v --timeout 300 --timeout-method thread -k "pw_cm or cm_mfma or adam or golden or bwd"
run pw_cm 300 python -u tools/studies/pw_cm_bench.py --reps 100
run pw_cm_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/pw_cm_stats -o run -- python3 tools/studies/pw_cm_bench.py --reps 50 --forms mfma
rm -f $OUT/pw_cm_stats/run_kernel_trace.csv
run ada_tune 300 python -u tools/studies/ada_bwd_tune.py
AIMET_ADA_PW_CM_FUSED=1 run ada2k_cm 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000

#!/usr/bin/env bash
# Round 4, session n: v3 channel-major MFMA kernels (operands loaded in the MFMA register layout,
# no LDS staging; 32-deep chunks double-buffered; targets prefetched) vs the library chain.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_pwcm 600 python -u -m pytest tests/test_gpu_parity.py tests/test_adaround_wrapper.py -v --timeout 300 --timeout-method thread -k "pw_cm or adam or cm_mfma or loop"
run pw_cm 300 python -u tools/studies/pw_cm_bench.py --reps 100
run pw_cm_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/pw_cm_stats -o run -- python3 tools/studies/pw_cm_bench.py --reps 50 --forms mfma
rm -f $OUT/pw_cm_stats/run_kernel_trace.csv
AIMET_ADA_PW_CM_FUSED=1 run ada2k_cm 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000

#!/usr/bin/env bash
# Round 4, session j: persistent fold partials for captured launches; k iterations per AdaRound
# graph; v2 MFMA channel-major kernels (split-K over waves, prefetched chunks) vs the library chain.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_ada 900 python -u -m pytest tests/test_adaround_wrapper.py tests/test_adaround_golden.py tests/test_adaround_dist_gpu.py -v --timeout 300 --timeout-method thread
run t_parity 900 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "adaround or learned_grid or lg_ or pw_cm"
run pw_cm 300 python -u tools/studies/pw_cm_bench.py
AIMET_ADA_GRAPH_ITERS=1 run ada2k_k1 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000
AIMET_ADA_GRAPH_ITERS=10 run ada2k_k10 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000
AIMET_ADA_PW_CM_FUSED=1 run ada2k_cm 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000
run lg16_trace 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lg16_trace -o run -- python3 benchmarks/lg16_roofline.py --reps 40
python tools/studies/lg16_trace_summary.py $OUT/lg16_trace r04 > $OUT/lg16_trace_summary.txt 2>&1

#!/usr/bin/env bash
# Round 4, session h: batched fold loads, dense-wave round pows, k iterations per AdaRound graph,
# MFMA channel-major kernels (off by default) measured against the library chain.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_parity 900 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "adaround or learned_grid or lg_ or search or calibrate or tfe or pw_cm"
run t_ada 900 python -u -m pytest tests/test_adaround_wrapper.py tests/test_adaround_golden.py tests/test_adaround_dist_gpu.py tests/test_llama_quantsim_gpu.py -v --timeout 300 --timeout-method thread
AIMET_ADA_BWD_U=1 run ada_tune_u1 300 python -u tools/studies/ada_bwd_tune.py
run lg16_trace 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lg16_trace -o run -- python3 benchmarks/lg16_roofline.py --reps 40
python tools/studies/lg16_trace_summary.py $OUT/lg16_trace r04 > $OUT/lg16_trace_summary.txt 2>&1
run pw_cm 300 python -u tools/studies/pw_cm_bench.py
run ada_trace 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/ada_trace -o run -- python3 benchmarks/adaround_mobilenet.py --iterations 300 --images 256
python tools/studies/ada_trace_summary.py $OUT/ada_trace 15900 $OUT/ada_trace_kernels.csv > $OUT/ada_trace_summary.txt 2>&1
run ada10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000
run bench 300 python -u bench.py

#!/usr/bin/env bash
# Round 4, session g: two-level arrival counters; range-gradient units against the exact sums of
# the fp32 terms; per-kernel rooflines; AdaRound loop (10k) and its trace.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_parity 900 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "adaround or learned_grid or lg_ or search or calibrate or tfe or pw_cm"
AIMET_BOUND_REPORT=$OUT/lg_bound_units.jsonl run t_lg 900 python -u -m pytest tests/test_range_learning.py tests/test_llama_quantsim_gpu.py tests/test_qat_ddp_gpu.py tests/test_adaround_golden.py tests/test_adaround_dist_gpu.py -v --timeout 300 --timeout-method thread
for u in 1 2; do
  AIMET_ADA_BWD_U=$u run ada_tune_u$u 300 python -u tools/studies/ada_bwd_tune.py
done
run lg16_bench 300 python -u benchmarks/lg16_roofline.py
run lg16_trace 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lg16_trace -o run -- python3 benchmarks/lg16_roofline.py --reps 40
python tools/studies/lg16_trace_summary.py $OUT/lg16_trace r04 > $OUT/lg16_trace_summary.txt 2>&1
run roofline 600 python -u benchmarks/kernel_roofline.py --no-cpu --out $OUT/kernel_roofline.jsonl
run ada_trace 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/ada_trace -o run -- python3 benchmarks/adaround_mobilenet.py --iterations 300 --images 256
python tools/studies/ada_trace_summary.py $OUT/ada_trace 15900 $OUT/ada_trace_kernels.csv > $OUT/ada_trace_summary.txt 2>&1
run ada10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000

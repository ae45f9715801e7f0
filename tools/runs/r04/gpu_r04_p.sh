#!/usr/bin/env bash
# Round 4, session p: channel-major weight gradient as a split-K batched GEMM; LG16 kernels with
# ping-pong buffers and unconditional prefetch (fold in kernel vs its own launch).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_ada 900 python -u -m pytest tests/test_adaround_wrapper.py tests/test_adaround_golden.py -v --timeout 300 --timeout-method thread
run t_lg 900 python -u -m pytest tests/test_gpu_parity.py tests/test_range_learning.py -v --timeout 300 --timeout-method thread -k "learned_grid or lg_ or range or adam or pw_cm"
run pw_cm 300 python -u tools/studies/pw_cm_bench.py --reps 100 --forms library
run lg16_fused 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lg16_fused -o run -- python3 benchmarks/lg16_roofline.py --reps 40
python tools/studies/lg16_trace_summary.py $OUT/lg16_fused r04_fused > $OUT/lg16_fused_summary.txt 2>&1
AIMET_LG_FOLD_LAUNCH=1 run lg16_launch 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lg16_launch -o run -- python3 benchmarks/lg16_roofline.py --reps 40
python tools/studies/lg16_trace_summary.py $OUT/lg16_launch r04_launch > $OUT/lg16_launch_summary.txt 2>&1
rm -f $OUT/lg16_fused/run_kernel_trace.csv $OUT/lg16_launch/run_kernel_trace.csv
run ada2k 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000
AIMET_ADA_CM_SPLITK=4 run ada2k_s4 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000

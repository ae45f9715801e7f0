#!/usr/bin/env bash
# Round 4, session q: the one-pass 1x1 step on the matrix cores (pw_mfma_step_kernel); the
# learned-grid per-tensor fold in two levels (group folds while the kernel streams).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_pw 600 python -u -m pytest tests/test_gpu_parity.py tests/test_adaround_wrapper.py -v --timeout 300 --timeout-method thread -k "pw_step or pw_fused or fused_step or loop or pw_cm"
run t_lg 900 python -u -m pytest tests/test_gpu_parity.py tests/test_range_learning.py tests/test_llama_quantsim_gpu.py tests/test_qat_ddp_gpu.py -v --timeout 300 --timeout-method thread -k "learned_grid or lg_ or range or llama or ddp"
run lg16_fused 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lg16_fused -o run -- python3 benchmarks/lg16_roofline.py --reps 40
python tools/studies/lg16_trace_summary.py $OUT/lg16_fused r04_fused2 > $OUT/lg16_fused_summary.txt 2>&1
AIMET_LG_FOLD_LAUNCH=1 run lg16_launch 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lg16_launch -o run -- python3 benchmarks/lg16_roofline.py --reps 40
python tools/studies/lg16_trace_summary.py $OUT/lg16_launch r04_launch2 > $OUT/lg16_launch_summary.txt 2>&1
rm -f $OUT/lg16_fused/run_kernel_trace.csv $OUT/lg16_launch/run_kernel_trace.csv
run ada2k 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000
AIMET_ADA_PW_MFMA=0 run ada2k_valu 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000

#!/usr/bin/env bash
# Round 4, session e: exhaustive sigmoid / reciprocal check; AdaRound backward with the faster
# sigmoid, wave-local compaction and the deterministic round loss; learned-grid per-tensor backward
# with the fold in the last workgroup.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run build_sig 300 hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -o /tmp/sigmoid_fast_check tools/studies/sigmoid_fast_check.hip
run sig_check 120 /tmp/sigmoid_fast_check
run t_ada 900 python -u -m pytest tests/test_adaround_golden.py tests/test_adaround_wrapper.py tests/test_adaround_dist_gpu.py -v --timeout 300 --timeout-method thread
run t_ada_parity 900 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "adaround or learned_grid or lg_"
run t_lg 900 python -u -m pytest tests/test_range_learning.py tests/test_llama_quantsim_gpu.py tests/test_qat_ddp_gpu.py -v --timeout 300 --timeout-method thread
for u in 1 2; do
  AIMET_ADA_BWD_U=$u run ada_tune_u$u 300 python -u tools/studies/ada_bwd_tune.py
done
run ada_pmc_valu 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $OUT/ada_pmc -o run -- python3 tools/studies/ada_bwd_tune.py --reps 1
run lg16_bench 300 python -u benchmarks/lg16_roofline.py
run lg16_trace 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lg16_trace -o run -- python3 benchmarks/lg16_roofline.py --reps 40
python tools/studies/lg16_trace_summary.py $OUT/lg16_trace r04 > $OUT/lg16_trace_summary.txt 2>&1

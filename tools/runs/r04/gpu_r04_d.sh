#!/usr/bin/env bash
# Round 4, session d: checkpoint tests (deterministic MIOpen), Llama range-gradient units, the
# wave-compacted AdaRound backward: bit-exact tests, U sweep, VALU counters.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
export AIMET_BOUND_REPORT=$OUT/lg_bound_units_llama.jsonl
rm -f $AIMET_BOUND_REPORT
run t_ckpt 600 python -u -m pytest tests/test_checkpoint.py -v --timeout 300 --timeout-method thread
AIMET_LG_BOUND_C=64 run t_llama 600 python -u -m pytest tests/test_llama_quantsim_gpu.py -v --timeout 300 --timeout-method thread
unset AIMET_BOUND_REPORT
run t_ada 900 python -u -m pytest tests/test_adaround_golden.py tests/test_adaround_wrapper.py tests/test_adaround_dist_gpu.py -v --timeout 300 --timeout-method thread
run t_ada_parity 900 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "adaround"
for u in 1 2 4; do
  AIMET_ADA_BWD_U=$u run ada_tune_u$u 300 python -u tools/studies/ada_bwd_tune.py
done
AIMET_ADA_BWD_U=2 run ada_pmc_valu 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $OUT/ada_pmc -o run -- python3 tools/studies/ada_bwd_tune.py --reps 1

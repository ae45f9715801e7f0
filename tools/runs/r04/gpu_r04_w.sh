#!/usr/bin/env bash
# Round 4, session w (run twice: w1 with both tail forms in one kernel -- SGPR spills, slower; w2 with a kernel-level TAIL flag): adaround_bwd_vec_kernel with the scalar-tail flags compile-time false on every
# tile but the last, lane masks from ballot_w64 and a one-instruction floor threshold -- rate and
# VALU count at 2^28 (checksums must equal profiles/r04/ada_bwd_tune_final.jsonl), the AdaRound tests.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
AIMET_ADA_BWD_U=1 run ada_tune_u1a 300 python -u tools/studies/ada_bwd_tune.py
AIMET_ADA_BWD_U=2 run ada_tune_u2 300 python -u tools/studies/ada_bwd_tune.py
AIMET_ADA_BWD_U=1 run ada_tune_u1b 300 python -u tools/studies/ada_bwd_tune.py
run ada_pmc_valu 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $OUT/ada_pmc -o run -- python3 tools/studies/ada_bwd_tune.py --reps 1
rm -f $OUT/ada_pmc/run_kernel_trace.csv
run t_ada 900 python -u -m pytest tests/test_adaround_wrapper.py tests/test_adaround_golden.py tests/test_adaround_dist_gpu.py tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -k "adaround or adam or dw or depthwise or pw_ or pointwise"

#!/usr/bin/env bash
# Round 6, session v: the AdaRound backward's base, rounding-loss gradient and dense pow in packed
# f32 (two elements per instruction): golden / parity, timing, counters.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
T="python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu"
run t_ada 600 $T tests/test_adaround_golden.py tests/test_gpu_parity.py -k "adaround"
run ada_tab 300 python tools/studies/ada_bwd_tune.py --scales 1,4 --tag v_pk
run ada_pmc 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/ada_pmc_v -o run -- python3 tools/studies/ada_bwd_tune.py --scales 1 --reps 1 --tag pmc_v
run ada_tab2 300 python tools/studies/ada_bwd_tune.py --scales 1,4 --tag v_pk_rep
run t_wrap 600 $T tests/test_adaround_wrapper.py tests/test_adaround_dist_gpu.py

#!/usr/bin/env bash
# Round 6, session g: the entropy search with parallel windows / selection; the AdaRound backward on the table-driven f32 pow (golden / parity / wrapper
# tests, exhaustive check against the Sleef emulation, 2^28 timing, counters, trace), the drop-in
# compute_encodings phases, the MSE / entropy search counters, then the default bench.py run.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
T="python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu"
run t_ada 600 $T tests/test_adaround_golden.py tests/test_gpu_parity.py -k "adaround"
run pow_check 300 tools/studies/pow_fast_check
run ada_tab 300 python tools/studies/ada_bwd_tune.py --scales 1,4 --tag r06_tab
run ada_reg0 300 python tools/studies/ada_bwd_tune.py --scales 1 --reg 0 --tag r06_tab_reg0
run ada_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ada_trace_tab -o run -- python3 tools/studies/ada_bwd_tune.py --scales 1 --tag trace_tab
run ada_pmc 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/ada_pmc_tab -o run -- python3 tools/studies/ada_bwd_tune.py --scales 1 --reps 1 --tag pmc_tab
run t_wrap 600 $T tests/test_adaround_wrapper.py
run t_ent 600 $T tests/test_entropy.py tests/test_search_resnet_gpu.py tests/test_gpu_parity.py -k "entropy or search or mse or calibrate or get_encodings"
run search_time 300 python tools/studies/tfe_search_time.py MSE ENTROPY
run dropin 300 python tools/studies/dropin_profile.py
P="--kernel-trace --output-format csv"
S="python3 tools/studies/tfe_search_time.py MSE ENTROPY"
run search_pmc_a 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU $P -d gpurun_out/search_pmc_a -o run -- $S
run search_pmc_b 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 $P -d gpurun_out/search_pmc_b -o run -- $S
run bench_full 660 python bench.py

#!/usr/bin/env bash
# Round 6, session d: config 1 sharded through the sim (MIOpen off in the worker), the MSE search
# with exact pruning vs the oracle, the f64 pow's exhaustive check against the Sleef emulation, and
# the per-channel searches' kernel times + counters.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
T="python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu"
run t_sharded 900 $T tests/test_quantsim_sharded_gpu.py
run t_search 900 $T tests/test_search_resnet_gpu.py
run t_parity 900 $T tests/test_gpu_parity.py -k "search or mse"
run pow_check 900 tools/studies/pow_fast_check
run search_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/search_trace2 -o run -- python3 tools/studies/tfe_search_time.py MSE ENTROPY
run search_pmc1 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d gpurun_out/search_pmc1 -o run -- python3 tools/studies/tfe_search_time.py MSE ENTROPY

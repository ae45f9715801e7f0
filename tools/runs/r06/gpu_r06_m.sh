#!/usr/bin/env bash
# Round 6, session m: the entropy search with the f32 filter (tests, timing, trace, counters).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
T="python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu"
run t_ent 600 $T tests/test_entropy.py tests/test_search_resnet_gpu.py tests/test_gpu_parity.py -k "entropy or search or mse or calibrate or get_encodings"
run search_time 300 python tools/studies/tfe_search_time.py MSE ENTROPY
run ent_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ent_trace_m -o run -- python3 tools/studies/tfe_search_time.py MSE ENTROPY
run ent_pmc 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d gpurun_out/ent_pmc_m -o run -- python3 tools/studies/tfe_search_time.py MSE ENTROPY
run ent_pmc_b 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 --kernel-trace --output-format csv -d gpurun_out/ent_pmc_mb -o run -- python3 tools/studies/tfe_search_time.py MSE ENTROPY
run knee 120 tools/studies/stream_pipe knee

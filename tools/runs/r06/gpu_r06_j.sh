#!/usr/bin/env bash
# Round 6, session j: config 5's QAT step, round-5 Python with this round's library vs both trees
# (which side holds the 14 ms / step difference); the entropy search with its own logarithm,
# level-wise normalisers (tests, timing, counters, step shares from study builds).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
T="python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu"
run t_ent 600 $T tests/test_entropy.py tests/test_search_resnet_gpu.py tests/test_gpu_parity.py -k "entropy or search or mse or calibrate or get_encodings"
run search_time 300 python tools/studies/tfe_search_time.py MSE ENTROPY
run ent_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ent_trace_j -o run -- python3 tools/studies/tfe_search_time.py ENTROPY
run ent_pmc 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d gpurun_out/ent_pmc_j -o run -- python3 tools/studies/tfe_search_time.py ENTROPY
run ent_no3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ent_no3_j -o run -- python3 tools/studies/tfe_search_time.py --lib tools/studies/ent_lib/no3/libaimet_amd.so ENTROPY
run ent_no23 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ent_no23_j -o run -- python3 tools/studies/tfe_search_time.py --lib tools/studies/ent_lib/no23/libaimet_amd.so ENTROPY
run llama_mix 600 python -u tools/studies/r05py_r06so/benchmarks/llama_qat.py --steps 5 --warmup 2
run llama_r06 600 python -u benchmarks/llama_qat.py --steps 5 --warmup 2
run llama_r05 600 python -u tools/studies/r05tree/benchmarks/llama_qat.py --steps 5 --warmup 2

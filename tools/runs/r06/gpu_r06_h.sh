#!/usr/bin/env bash
# Round 6, session h: the entropy search skipping empty bins' logarithms (segment-major items),
# the AdaRound backward's branch-free dense fast pow (tests, timing; U = 2 study build beside it),
# config 5 re-timed alone (quantsim and plain), the entropy counters.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
T="python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu"
run t_ada 600 $T tests/test_adaround_golden.py tests/test_gpu_parity.py -k "adaround"
run t_ent 600 $T tests/test_entropy.py tests/test_search_resnet_gpu.py tests/test_gpu_parity.py -k "entropy or search or mse or calibrate or get_encodings"
run search_time 300 python tools/studies/tfe_search_time.py MSE ENTROPY
run ada_tab 300 python tools/studies/ada_bwd_tune.py --scales 1,4 --tag r06_tab_bf
run ada_u2 300 python tools/studies/ada_bwd_tune.py --scales 1,4 --tag r06_tab_bf_u2 --lib tools/studies/lib_u2/libaimet_amd.so
run ada_tab2 300 python tools/studies/ada_bwd_tune.py --scales 1,4 --tag r06_tab_bf_rep
run search_pmc_a 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d gpurun_out/search_pmc_h -o run -- python3 tools/studies/tfe_search_time.py ENTROPY
run llama 600 python -u benchmarks/llama_qat.py --steps 5 --warmup 2
run llama_plain 600 python -u benchmarks/llama_qat.py --steps 5 --warmup 2 --path plain
run ent_no3 300 python tools/studies/tfe_search_time.py --lib tools/studies/ent_lib/no3/libaimet_amd.so ENTROPY
run ent_no23 300 python tools/studies/tfe_search_time.py --lib tools/studies/ent_lib/no23/libaimet_amd.so ENTROPY
run ent_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ent_trace_h -o run -- python3 tools/studies/tfe_search_time.py MSE ENTROPY

#!/usr/bin/env bash
# Round 6, session i: config 5 on the round-5 tree vs this tree on the same box (the QAT step read
# 250 ms this round against 229 in round 5); the entropy search's step shares from study builds
# under the kernel tracer; whether software pipelining hides the AdaRound backward's arithmetic.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run llama_r05 600 python -u tools/studies/r05tree/benchmarks/llama_qat.py --steps 5 --warmup 2
run llama_r06 600 python -u benchmarks/llama_qat.py --steps 5 --warmup 2
run llama_r05b 600 python -u tools/studies/r05tree/benchmarks/llama_qat.py --steps 5 --warmup 2
run stream_pipe 300 tools/studies/stream_pipe
run ent_no3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ent_no3 -o run -- python3 tools/studies/tfe_search_time.py --lib tools/studies/ent_lib/no3/libaimet_amd.so ENTROPY
run ent_no23 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ent_no23 -o run -- python3 tools/studies/tfe_search_time.py --lib tools/studies/ent_lib/no23/libaimet_amd.so ENTROPY

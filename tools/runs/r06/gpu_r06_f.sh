#!/usr/bin/env bash
# Round 6, session f: the default bench.py run (headline + configs 3 / 5 secondaries, wall-clock
# timed as the driver sees it), the drop-in compute_encodings phases, and the MSE / entropy search
# counters (VALU per candidate x bin) on ResNet-50's 27,560 channels.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run bench_full 700 python bench.py
run dropin 300 python tools/studies/dropin_profile.py
P="--kernel-trace --output-format csv"
S="python3 tools/studies/tfe_search_time.py MSE ENTROPY"
run search_pmc_a 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU $P -d gpurun_out/search_pmc_a -o run -- $S
run search_pmc_b 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 $P -d gpurun_out/search_pmc_b -o run -- $S

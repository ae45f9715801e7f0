#!/usr/bin/env bash
# Round 6, session aa: LDS counters of the AdaRound backward (bank conflicts of the pow tables'
# per-lane gathers).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_lds 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/ada_lds -o run -- python3 tools/studies/ada_bwd_tune.py --scales 1 --reps 1 --tag lds

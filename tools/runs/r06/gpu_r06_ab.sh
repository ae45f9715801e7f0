#!/usr/bin/env bash
# Round 6, session ab: the fast pow's LDS tables as planar arrays (product) against the packed
# 16-B / 8-B entries (study build): parity, timing (alternating), bank-conflict counters.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
T="python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu"
run t_ada 600 $T tests/test_adaround_golden.py tests/test_gpu_parity.py -k "adaround"
A=tools/studies/ada_lib/aos/libaimet_amd.so
run tab_pl1 300 python tools/studies/ada_bwd_tune.py --scales 1,4 --tag planar
run tab_aos1 300 python tools/studies/ada_bwd_tune.py --scales 1,4 --tag aos --lib $A
run tab_pl2 300 python tools/studies/ada_bwd_tune.py --scales 1,4 --tag planar
run tab_aos2 300 python tools/studies/ada_bwd_tune.py --scales 1,4 --tag aos --lib $A
run ada_lds 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/ada_lds_pl -o run -- python3 tools/studies/ada_bwd_tune.py --scales 1 --reps 1 --tag lds_planar

#!/usr/bin/env bash
# Round 5, session ak: the stream shape again with one tile per workgroup beside the 8192-workgroup
# grid stride (tools/studies/stream_mix.hip), and the AdaRound backward without the loss value
# launched one tile per workgroup (a temporary build, -DADA_FULL_GRID=1, exp_libs/lib_full.so).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run stream_mix2 300 tools/studies/stream_mix
run ada_full 300 python -u tools/studies/ada_bwd_tune.py --lib tools/studies/exp_libs/lib_full.so --tag full_grid
run ada_base_c 300 python -u tools/studies/ada_bwd_tune.py --tag base
run ada_full0 300 python -u tools/studies/ada_bwd_tune.py --reg 0 --lib tools/studies/exp_libs/lib_full.so --tag full_grid_reg0
run ada_full_b 300 python -u tools/studies/ada_bwd_tune.py --lib tools/studies/exp_libs/lib_full.so --tag full_grid

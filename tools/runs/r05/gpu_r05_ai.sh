#!/usr/bin/env bash
# Round 5, session ai: the AdaRound backward with the next tile's loads issued before the current
# tile's arithmetic (a temporary build, -DADA_BWD_PF=1, tools/studies/exp_libs/lib_pf.so) beside the
# library's form, with and without the rounding loss; checksums must agree.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_base 300 python -u tools/studies/ada_bwd_tune.py --tag base
run ada_pf 300 python -u tools/studies/ada_bwd_tune.py --lib tools/studies/exp_libs/lib_pf.so --tag pf
run ada_base0 300 python -u tools/studies/ada_bwd_tune.py --reg 0 --tag base_reg0
run ada_pf0 300 python -u tools/studies/ada_bwd_tune.py --reg 0 --lib tools/studies/exp_libs/lib_pf.so --tag pf_reg0
grep -h '^{' $OUT/ada_base.log $OUT/ada_pf.log $OUT/ada_base0.log $OUT/ada_pf0.log > $OUT/ada_pf.jsonl

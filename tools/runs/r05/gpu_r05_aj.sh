#!/usr/bin/env bash
# Round 5, session aj: the HBM rate of the AdaRound backward's stream shape (3 reads + 1 write) with
# and without arithmetic and with the buffers' starts skewed (tools/studies/stream_mix.hip); the
# backward itself with skewed buffers; and the prefetching build (lib_pf.so) again, run first this time.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run stream_mix 300 tools/studies/stream_mix
run ada_pf_b 300 python -u tools/studies/ada_bwd_tune.py --lib tools/studies/exp_libs/lib_pf.so --tag pf
run ada_base_b 300 python -u tools/studies/ada_bwd_tune.py --tag base
run ada_skew 300 python -u tools/studies/ada_bwd_tune.py --skew 4352 --tag skew4352
run ada_skew0 300 python -u tools/studies/ada_bwd_tune.py --reg 0 --skew 4352 --tag skew4352_reg0
run ada_skew2m 300 python -u tools/studies/ada_bwd_tune.py --reg 0 --skew $(( (2 << 20) + 4352 )) --tag skew2m_reg0

#!/usr/bin/env bash
# Round 5, session ar: the dense waves' pows without a branch per pair (a temporary build,
# -DADA_DENSE_ILP=1, exp_libs/lib_ilp.so: the pairs' chains in one block) beside the library's
# form at 2^28; checksums must agree.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_base_d 300 python -u tools/studies/ada_bwd_tune.py --tag base
run ada_ilp 300 python -u tools/studies/ada_bwd_tune.py --tag dense_ilp --lib tools/studies/exp_libs/lib_ilp.so
run ada_base_e 300 python -u tools/studies/ada_bwd_tune.py --tag base
run ada_ilp_b 300 python -u tools/studies/ada_bwd_tune.py --tag dense_ilp --lib tools/studies/exp_libs/lib_ilp.so
grep -h '^{' $OUT/ada_base_d.log $OUT/ada_ilp.log $OUT/ada_base_e.log $OUT/ada_ilp_b.log > $OUT/ada_dense_ilp.jsonl

#!/usr/bin/env bash
# Round 5, session am: the learned-grid forward of float32 weights cast to bf16 (the Llama-3-8B
# W4A16 weight path) at Llama-3-8B's weight shapes: the library's form (two quads per lane, 8-B
# stores) beside temporary builds with 8 consecutive elements per group and one 16-B store
# (-DLG_FWD8=G, G groups per lane: exp_libs/lib_fwd8_g{1,2}.so); checksums must agree.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run lgf_base 300 python -u tools/studies/lg_fwd_tune.py --tag base
run lgf_g1 300 python -u tools/studies/lg_fwd_tune.py --tag fwd8_g1 --lib tools/studies/exp_libs/lib_fwd8_g1.so
run lgf_g2 300 python -u tools/studies/lg_fwd_tune.py --tag fwd8_g2 --lib tools/studies/exp_libs/lib_fwd8_g2.so
run lgf_base_b 300 python -u tools/studies/lg_fwd_tune.py --tag base
run lgf_f32 300 python -u tools/studies/lg_fwd_tune.py --tag base --out f32
grep -h '^{' $OUT/lgf_*.log > $OUT/lg_fwd_tune.jsonl

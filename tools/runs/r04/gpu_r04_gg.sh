#!/usr/bin/env bash
# Round 4, session gg: what the weights cost a compute_encodings call -- both / activations only /
# weights only, reset-and-recompute medians (tools/studies/enc_split_cost.py).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run enc_split 300 python -u tools/studies/enc_split_cost.py

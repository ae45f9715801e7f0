#!/usr/bin/env bash
# Round 5, session ad: StatsBatch with and without the copy on a network with in-place ops.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run sb_inplace 300 python -u tools/studies/statsbatch_inplace_check.py

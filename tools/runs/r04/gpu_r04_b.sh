#!/usr/bin/env bash
# Round 4, session b: checkpoint debug
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ckpt_debug 300 python -u tools/studies/ckpt_debug.py

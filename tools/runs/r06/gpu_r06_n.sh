#!/usr/bin/env bash
# Round 6, session n: the full GPU test suite at this tree, then the search phases (where the
# getEncodings wall-clock beyond the kernels goes) and the stream's arithmetic knee.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run gpu_suite 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread
run search_phases 300 python tools/studies/tfe_search_time.py MSE ENTROPY
run knee 120 tools/studies/stream_pipe knee

#!/usr/bin/env bash
# Round 5, session ag: the default bench line after the secondary measurements were guarded.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run bench1 600 python -u bench.py

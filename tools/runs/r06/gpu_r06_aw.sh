#!/usr/bin/env bash
# Round 6, session aw: every hot-path kernel's roofline at the final tree (2^28 elements, HIP events
# over 10 launches; no CPU column), benchmarks/kernel_roofline.py.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run roofline 600 python -u benchmarks/kernel_roofline.py --no-cpu --out gpurun_out/kernel_roofline_r06.jsonl

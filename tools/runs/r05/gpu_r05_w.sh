#!/usr/bin/env bash
# Round 5, session w: the calibration plan with the entropy analyzer too -- single device (per-tensor
# and per-channel) and sharded over 2 gloo ranks / a world-size-1 RCCL group.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_plan_ent 600 python -u -m pytest tests/test_gpu_parity.py tests/test_distributed_gpu.py -v --timeout 300 --timeout-method thread -k "plan"

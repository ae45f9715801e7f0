#!/usr/bin/env bash
# Round 4, session o: the channel-major MFMA forward taken apart (tools/studies/pw_cm_probe.hip).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
mkdir -p /tmp/probe && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -o /tmp/probe/pw_cm_probe tools/studies/pw_cm_probe.hip
run pw_probe 120 /tmp/probe/pw_cm_probe

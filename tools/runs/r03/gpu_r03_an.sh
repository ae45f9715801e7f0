#!/usr/bin/env bash
# Round 3: host split of the native compute_encodings call.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run enc_host 300 python -u tools/studies/enc_native_host.py

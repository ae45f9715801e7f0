#!/usr/bin/env bash
# Round 5, session x: where the drop-in QuantizationSimModel.compute_encodings spends its time.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run dropin_prof 300 python -u tools/studies/dropin_profile.py --reps 3

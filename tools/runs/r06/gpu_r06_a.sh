#!/usr/bin/env bash
# Round 6, session a: the round-5 tree on a fresh box -- smoke, the default bench line, the drop-in
# compute_encodings profile (the starting point of the round's drop-in work).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py
run dropin 300 python tools/studies/dropin_profile.py --reps 3

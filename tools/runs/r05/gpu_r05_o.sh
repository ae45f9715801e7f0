#!/usr/bin/env bash
# Round 5, session o: exhaustive check of the certified f64 pow (tools/studies/pow_cert_check.hip)
# -- a short pass over 256 exponents, then every exponent of the list.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run cert_short 180 tools/studies/pow_cert_check 256
if grep -q "certified but != pow01_log: 0" $OUT/cert_short.log; then
  run cert_full 1000 tools/studies/pow_cert_check
fi

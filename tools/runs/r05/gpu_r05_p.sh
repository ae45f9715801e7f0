#!/usr/bin/env bash
# Round 5, session p: VALU issue rates of f32 / packed f32 / f64 FMA and f32<->f64 conversions.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run valu_rates 120 tools/studies/valu_rates

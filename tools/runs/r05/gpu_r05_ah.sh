#!/usr/bin/env bash
# Round 5, session ah: the AdaRound backward without the rounding loss (reg 0: no pow) beside the
# loop's form, and its VALU per element -- how much of the kernel the exact pow is.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_reg0 300 python -u tools/studies/ada_bwd_tune.py --reg 0 --tag reg0
run ada_reg 300 python -u tools/studies/ada_bwd_tune.py --tag reg0.01
run ada_pmc0 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $OUT/ada_pmc0 -o run -- python3 tools/studies/ada_bwd_tune.py --reps 1 --reg 0
python3 - <<'PY' > $OUT/ada_bwd_valu_reg0.txt 2>&1
import csv, glob
f = glob.glob("gpurun_out/ada_pmc0/*counter_collection.csv")[0]
rows = [r for r in csv.DictReader(open(f)) if "adaround_bwd_vec_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "SQ_INSTS_VALU"]
for r in rows:
    print(r["Kernel_Name"][:90], r["Counter_Value"], round(float(r["Counter_Value"]) * 64 / 2**28, 1), "VALU per element")
PY
rm -rf $OUT/ada_pmc0

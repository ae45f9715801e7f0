#!/usr/bin/env bash
# Round 5, session k: the AdaRound backward's dense waves evaluating their pows two at a time in
# packed f32 -- golden parity, the 2^28 kernel rate, VALU per element (SQ_INSTS_VALU).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run t_ada 600 python -u -m pytest tests/test_adaround_golden.py tests/test_adaround_wrapper.py -q --timeout 300 --timeout-method thread
run ada_tune 300 python -u tools/studies/ada_bwd_tune.py --tag packed_dense
run ada_pmc_valu 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $OUT/ada_pmc -o run -- python3 tools/studies/ada_bwd_tune.py --reps 1
python3 - <<'PY' > $OUT/ada_bwd_valu.txt 2>&1
import csv, glob
f = glob.glob("gpurun_out/ada_pmc/*counter_collection.csv")[0]
rows = [r for r in csv.DictReader(open(f)) if "adaround_bwd_vec_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "SQ_INSTS_VALU"]
for r in rows:
    print(r["Kernel_Name"][:90], r["Counter_Value"], round(float(r["Counter_Value"]) * 64 / 2**28, 1), "VALU per element")
PY
rm -rf $OUT/ada_pmc

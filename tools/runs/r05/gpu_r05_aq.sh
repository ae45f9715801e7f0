#!/usr/bin/env bash
# Round 5, session aq (the final tree, one tile per workgroup without the loss value): where the AdaRound backward's wave time goes (issue vs park vs stall) and the
# effective clock it runs at -- two PMC passes over tools/studies/ada_bwd_tune.py --reps 1.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run pmc_a_final 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/ada_pmc_a -o run -- python3 tools/studies/ada_bwd_tune.py --reps 1
run pmc_b_final 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d $OUT/ada_pmc_b -o run -- python3 tools/studies/ada_bwd_tune.py --reps 1
python3 - <<'PY' > $OUT/ada_bwd_pmc_final.txt 2>&1
import csv, glob, collections
for tag in ("a", "b"):
    for f in glob.glob(f"gpurun_out/ada_pmc_{tag}/*counter_collection.csv"):
        acc = collections.OrderedDict()
        for r in csv.DictReader(open(f)):
            if "adaround_bwd_vec_kernel" not in r["Kernel_Name"]:
                continue
            key = (r["Dispatch_Id"], r["Kernel_Name"][:70])
            acc.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
        for (d, k), v in acc.items():
            print(tag, d, k, " ".join(f"{n}={x:.0f}" for n, x in sorted(v.items())))
    for f in glob.glob(f"gpurun_out/ada_pmc_{tag}/*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            if "adaround_bwd_vec_kernel" in r["Kernel_Name"]:
                print(tag, "trace", r["Dispatch_Id"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, "ms")
PY
rm -rf $OUT/ada_pmc_a $OUT/ada_pmc_b

"""Memory copies around the second-to-last occurrence of a kernel (rocprofv3 --memory-copy-trace):
python3 tools/studies/copy_timeline.py <trace_dir> [anchor]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "minmax_many_kernel"
k = sorted(csv.DictReader(open(glob.glob(os.path.join(d, "*kernel_trace.csv"))[0])),
           key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(k) if anchor in r["Kernel_Name"]]
t0 = int(k[idx[-2] if len(idx) > 1 else idx[-1]]["Start_Timestamp"])
f = glob.glob(os.path.join(d, "*memory_copy_trace.csv"))
rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Start_Timestamp"])) if f else []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if -3e6 < s - t0 < 8e6:
        print("%9.1f %8.1f us %s %s B" % ((s - t0) / 1e3, (e - s) / 1e3, r.get("Direction", "?"), r.get("Bytes", "?")))

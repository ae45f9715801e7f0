"""Print the kernel timeline (start offset, duration, queue) around the last occurrence of a kernel
in a rocprofv3 --kernel-trace CSV: python3 tools/studies/trace_timeline.py run_kernel_trace.csv [anchor] [before] [after]"""
import csv
import sys

path = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "minmax_many_kernel"
before = int(sys.argv[3]) if len(sys.argv) > 3 else 8
after = int(sys.argv[4]) if len(sys.argv) > 4 else 20
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
i0 = idx[-2] if len(idx) > 1 else idx[-1]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[max(0, i0 - before):i0 + after]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("aimet_amd::(anonymous namespace)::", "")
    print("%9.1f %8.1f us q%-3s %s" % ((s - t0) / 1e3, (e - s) / 1e3, r["Queue_Id"], name[:90]))

"""Per-kernel mean duration of benchmarks/lg16_roofline.py's calls from a rocprofv3 kernel trace:
the 16-bit learned-grid forward / backward kernels and the torch copy / add controls, one line per
(kernel, problem size) in the order they ran, with the bytes each moved per element.

usage: python tools/studies/lg16_trace_summary.py <trace_dir> [label]"""
import csv
import glob
import json
import os
import sys

SIZES = {2048 * 4096: "seq2048x4096", 13_688_832: "mean_call", 2048 * 14336: "seq2048x14336",
         2048 * 1024: "seq2048x1024"}
KINDS = (("lg_fwd16_kernel", "fwd16", 4), ("lg_bwd16_tensor_kernel", "bwd16", 6), ("lg_bwd_fold_one", "fold", 0),
         ("copy", "copy", 4), ("add", "add", 6))


def main():
    path = sys.argv[1]
    label = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(path.rstrip("/"))
    files = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    rows = sorted(csv.DictReader(open(files[0])), key=lambda r: int(r["Start_Timestamp"]))
    # the benchmark times 1 + reps back-to-back calls of fwd, bwd (+ its fold), copy, add per size:
    # runs of one kernel kind of >= 20 calls, 4 per size in the benchmark's order of sizes (the
    # tensor set-up kernels between them form short runs and are dropped)
    order = list(SIZES.values())
    runs = []
    for r in rows:
        name = r["Kernel_Name"]
        kind = next((k[1] for k in KINDS if k[0] in name), "other")
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if kind == "fold" and runs and runs[-1]["kind"] == "bwd16":
            runs[-1]["fold"].append(us)
            continue
        if not runs or runs[-1]["kind"] != kind:
            runs.append({"kind": kind, "us": [], "fold": []})
        runs[-1]["us"].append(us)
    runs = [r for r in runs if len(r["us"]) >= 20 and r["kind"] != "other"]
    groups, seen = {}, []
    for i, r in enumerate(runs):
        size = order[min(i // 4, len(order) - 1)]
        for kind, us in ((r["kind"], r["us"]), ("fold", r["fold"])):
            if us:
                groups[(kind, size)] = us
                seen.append((kind, size))
    elems = {v: k for k, v in SIZES.items()}
    bpe = {k[1]: k[2] for k in KINDS}
    for key in seen:
        d = groups[key][1:] or groups[key]   # the first call of each (cold) dropped
        us = sum(d) / len(d)
        nb = bpe[key[0]] * elems[key[1]]
        print(json.dumps({"label": label, "kernel": key[0], "size": key[1], "calls": len(d), "mean_us": round(us, 2),
                          "TBps": round(nb / us / 1e6, 3) if nb else None}))


if __name__ == "__main__":
    main()

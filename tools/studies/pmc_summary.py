"""Compact summary of rocprofv3 --pmc counter CSVs: one line per (kernel, distinct counter set), the
first dispatch of each, with per-unit ratios when the unit count is given.

    python tools/studies/pmc_summary.py DIR [--match SUBSTR] [--units N] [--unit-name elem]

`units` divides the wave-instruction counters by N / 64 (per-lane work units: SQ_INSTS_* count
wave instructions, one per 64 lanes), e.g. --units 268435456 for the AdaRound backward at 2^28
elements. Also prints the kernel-trace durations of the same kernels when the trace CSV is there.
"""
import argparse
import collections
import csv
import glob
import os


def _short(name):
    name = name.replace("void ", "").replace("aimet_amd::(anonymous namespace)::", "")
    return name.split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    ap.add_argument("--units", type=float, default=0.0)
    ap.add_argument("--unit-name", default="unit")
    args = ap.parse_args()
    (path,) = glob.glob(os.path.join(args.dir, "*counter_collection.csv"))
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if args.match not in r["Kernel_Name"]:
            continue
        key = (int(r["Dispatch_Id"]), r["Kernel_Name"])
        disp.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    seen = set()
    for (d, name), c in disp.items():
        # one line per kernel and instruction mix (repeated dispatches differ only in cycles)
        sig = (name, tuple(sorted((k, v) for k, v in c.items() if k.startswith("SQ_INSTS") or k == "SQ_WAVES")))
        if sig in seen:
            continue
        seen.add(sig)
        short = _short(name)
        print("dispatch %d  %s" % (d, short))
        for k, v in sorted(c.items()):
            line = "    %-26s %16.0f" % (k, v)
            if args.units and k.startswith("SQ_INSTS"):
                line += "   %.2f per %s" % (v / (args.units / 64.0), args.unit_name)
            print(line)
        if "SQ_WAVE_CYCLES" in c and "SQ_INSTS_VALU" in c and c["SQ_WAVE_CYCLES"]:
            print("    VALU instructions per wave-cycle: %.3f" % (c["SQ_INSTS_VALU"] / c["SQ_WAVE_CYCLES"]))
    tr = glob.glob(os.path.join(args.dir, "*kernel_trace.csv"))
    if tr:
        dur = collections.defaultdict(list)
        for r in csv.DictReader(open(tr[0])):
            if args.match in r["Kernel_Name"]:
                dur[_short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        for k, v in dur.items():
            print("trace %s: %d dispatches, median %.3f ms (under the counters)" % (k, len(v), sorted(v)[len(v) // 2]))


if __name__ == "__main__":
    main()

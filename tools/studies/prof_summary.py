"""Summarise a rocprofv3 kernel trace (+ optional FETCH_SIZE / WRITE_SIZE PMC passes) of bench.py.

usage: python tools/studies/prof_summary.py <trace_dir> [<pmc_fetch_dir> <pmc_write_dir>] [--steps N]
Prints per-kernel totals over the timed steps and, with PMC data, the HBM bytes per step of the
per-tensor QDQ kernel corrected as MI355X_MICROARCH.md §HBM prescribes (FETCH_SIZE x 2 on gfx950,
WRITE_SIZE as is; both in KiB).
"""
import collections
import csv
import glob
import os
import sys

QDQ = "tensor_vec_kernel"


def trace_rows(d):
    f = glob.glob(os.path.join(d, "*kernel_trace.csv"))[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def pmc(d, name):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    return [(r["Kernel_Name"], float(r["Counter_Value"])) for r in csv.DictReader(open(f)) if r["Counter_Name"] == name]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    per_step = 55
    rows = trace_rows(args[0])
    qi = [i for i, r in enumerate(rows) if QDQ in r["Kernel_Name"]]
    # skip warmup: use the last 5 steps of QDQ dispatches
    nsteps = len(qi) // per_step
    first = qi[(nsteps - min(nsteps, 5)) * per_step]
    ai = [i for i, r in enumerate(rows) if "aimet_amd" in r["Kernel_Name"]]
    seg = rows[first:ai[-1] + 1]
    steps = min(nsteps, 5)
    agg = collections.defaultdict(lambda: [0, 0])
    for r in seg:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-60:]
        agg[k][0] += 1
        agg[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    span = int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])
    print("timed steps analysed: %d, span %.3f ms/step" % (steps, span / 1e6 / steps))
    for k, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print("  %-62s calls/step %5.1f  ms/step %.4f" % (k, c / steps, d / 1e6 / steps))
    q_ns = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg if QDQ in r["Kernel_Name"]) / steps
    print("per-tensor QDQ kernel time/step: %.4f ms" % (q_ns / 1e6))
    # calibration (compute_encodings) = every aimet kernel before the first QDQ dispatch
    cal = [r for r in rows[:qi[0]] if "aimet_amd" in r["Kernel_Name"]]
    if cal:
        cagg = collections.defaultdict(lambda: [0, 0])
        for r in cal:
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("aimet_amd::", "")
            k = k.replace("void ", "").split("(")[0][-60:]
            cagg[k][0] += 1
            cagg[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        tot = sum(d for _, d in cagg.values())
        # bench.py runs compute_encodings 1 + --enc-reps times: one minmax_many launch per call
        ncalls = max(1, sum(c for k, (c, _) in cagg.items() if k.startswith("minmax_many_kernel")))
        # kernels of the parameter stream overlap the activation passes: also report the union of
        # the busy intervals (the GPU time a call actually occupies)
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in cal)
        busy, cs, ce = 0, iv[0][0], iv[0][1]
        for s0, e0 in iv[1:]:
            if s0 > ce:
                busy += ce - cs
                cs, ce = s0, e0
            else:
                ce = max(ce, e0)
        busy += ce - cs
        print("compute_encodings kernels (before the first QDQ step): %d calls, %.3f ms summed kernel time per "
              "call, %.3f ms GPU busy per call (union of overlapping kernels)"
              % (ncalls, tot / 1e6 / ncalls, busy / 1e6 / ncalls))
        for k, (c, d) in sorted(cagg.items(), key=lambda x: -x[1][1]):
            print("  %-62s calls/call %4.1f  ms/call %.4f  avg us %.1f" % (k, c / ncalls, d / 1e6 / ncalls,
                                                                         d / 1e3 / c))
    if len(args) >= 3:
        f = [v for n, v in pmc(args[1], "FETCH_SIZE") if QDQ in n][-per_step:]
        w = [v for n, v in pmc(args[2], "WRITE_SIZE") if QDQ in n][-per_step:]
        fb, wb = sum(f) * 1024 * 2, sum(w) * 1024
        print("per-tensor QDQ HBM traffic/step: fetch %.4f GB (FETCH_SIZE x2), write %.4f GB, total %.4f GB"
              % (fb / 1e9, wb / 1e9, (fb + wb) / 1e9))
        # calibration kernels: every dispatch before the first QDQ one (one compute_encodings)
        fa, wa = pmc(args[1], "FETCH_SIZE"), pmc(args[2], "WRITE_SIZE")
        cut_f = next(i for i, (n, _) in enumerate(fa) if QDQ in n)
        cut_w = next(i for i, (n, _) in enumerate(wa) if QDQ in n)
        cf, cw = collections.defaultdict(float), collections.defaultdict(float)
        for n, v in fa[:cut_f]:
            if "aimet_amd" in n:
                cf[n.replace("(anonymous namespace)::", "").replace("aimet_amd::", "").replace("void ", "")
                   .split("(")[0]] += v * 1024 * 2
        for n, v in wa[:cut_w]:
            if "aimet_amd" in n:
                cw[n.replace("(anonymous namespace)::", "").replace("aimet_amd::", "").replace("void ", "")
                   .split("(")[0]] += v * 1024
        nc = max(1, sum(1 for n, _ in fa[:cut_f] if "minmax_many_kernel" in n))
        print("compute_encodings HBM traffic per kernel per call (FETCH_SIZE x2 + WRITE_SIZE; %d calls):" % nc)
        for k in sorted(cf, key=lambda k: -cf[k]):
            print("  %-62s fetch %.4f GB  write %.4f GB" % (k, cf[k] / 1e9 / nc, cw.get(k, 0) / 1e9 / nc))


if __name__ == "__main__":
    main()

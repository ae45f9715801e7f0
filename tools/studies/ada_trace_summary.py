"""Per-kernel split of the AdaRound optimisation loop from a rocprofv3 kernel trace.

usage: python tools/studies/ada_trace_summary.py <trace_dir> <layer_iterations> [out.csv]
Each layer's loop window runs from its first to its last aimet_amd adaround kernel (windows are
split where consecutive adaround kernels are more than 20 ms apart: the next layer's activation
caching runs there); every kernel inside a window is summed by name and divided by the number of
layer-iterations (layers x iterations per layer)."""
import collections
import csv
import glob
import os
import sys


def main():
    d, n_it = sys.argv[1], int(sys.argv[2])
    out = sys.argv[3] if len(sys.argv) > 3 else None
    f = glob.glob(os.path.join(d, "*kernel_trace.csv"))[0]
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f))]
    rows.sort()
    ada = [r for r in rows if "adaround_" in r[2]]
    windows = [[ada[0][0], ada[0][1]]]
    for s, e, _ in ada[1:]:
        if s - windows[-1][1] > 20_000_000:
            windows.append([s, e])
        else:
            windows[-1][1] = max(windows[-1][1], e)
    tot, cnt = collections.Counter(), collections.Counter()
    w = 0
    for s, e, n in rows:
        while w < len(windows) and s > windows[w][1]:
            w += 1
        if w == len(windows):
            break
        if s >= windows[w][0] and e <= windows[w][1]:
            tot[n] += e - s
            cnt[n] += 1
    busy = sum(tot.values())
    span = sum(b - a for a, b in windows)
    print("%d layer windows, %.1f ms, kernel busy %.1f ms (%.1f%%), %d layer-iterations: %.1f us window / %.1f us "
          "busy per layer-iteration" % (len(windows), span / 1e6, busy / 1e6, 100 * busy / span, n_it,
                                        span / 1e3 / n_it, busy / 1e3 / n_it))
    lines = []
    for n, t in tot.most_common():
        lines.append((n, cnt[n], t / 1e6, t / 1e3 / n_it, 100 * t / busy))
    for n, c, ms, us, pct in lines[:25]:
        print("%9.1f ms %7d calls %8.2f us/layer-it %5.1f%%  %s" % (ms, c, us, pct, n[:100]))
    if out:
        with open(out, "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["kernel", "calls", "total_ms", "us_per_layer_iteration", "pct_of_loop_busy"])
            for n, c, ms, us, pct in lines:
                w.writerow([n, c, round(ms, 3), round(us, 3), round(pct, 2)])


if __name__ == "__main__":
    main()

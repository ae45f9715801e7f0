"""Timeline of one compute_encodings call from a rocprofv3 trace of bench.py: every calibration
kernel of the last call before the first QDQ step, with its start / end relative to the call's
first kernel (us) and its queue, so the critical path and the gaps between launches can be read
off. With a HIP API trace in the same directory (--hip-runtime-trace) the host's calls of that
call are listed on the same clock: from the synchronize that opens bench.py's timed region to the
wait that ends it.

usage: python tools/studies/enc_timeline.py <trace_dir>
"""
import csv
import glob
import os
import sys

QDQ = "tensor_vec_kernel"


def short(name):
    k = name.replace("(anonymous namespace)::", "").replace("aimet_amd::", "")
    return k.replace("void ", "").split("(")[0][-58:]


def main():
    f = glob.glob(os.path.join(sys.argv[1], "*kernel_trace.csv"))[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    q0 = next(i for i, r in enumerate(rows) if QDQ in r["Kernel_Name"])
    cal = [r for r in rows[:q0] if "aimet_amd" in r["Kernel_Name"]]
    starts = [i for i, r in enumerate(cal) if "minmax_many_kernel" in r["Kernel_Name"]]
    first = starts[-1]
    while first > 0 and int(cal[first]["Start_Timestamp"]) - int(cal[first - 1]["End_Timestamp"]) < 200_000 \
            and "tfe_search" not in cal[first - 1]["Kernel_Name"]:
        first -= 1
    seg = cal[first:]
    t0 = int(seg[0]["Start_Timestamp"])
    t_end = max(int(r["End_Timestamp"]) for r in seg)
    qcol = next((c for c in ("Queue_Id", "Stream_Id", "Queue_ID") if c in seg[0]), None)
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + short(r["Kernel_Name"]),
           r.get(qcol, "?") if qcol else "?") for r in seg]
    api = glob.glob(os.path.join(sys.argv[1], "*hip_api_trace.csv"))
    if api:
        calls = sorted(csv.DictReader(open(api[0])), key=lambda r: int(r["Start_Timestamp"]))
        syncs = [int(r["Start_Timestamp"]) for r in calls
                 if r["Function"] in ("hipDeviceSynchronize", "hipStreamSynchronize") and int(r["Start_Timestamp"]) < t0]
        a0 = syncs[-1] if syncs else t0 - 2_000_000
        for r in calls:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if a0 <= s <= t_end + 1_000_000:
                ev.append((s, e, "H " + r["Function"], "host"))
        t0 = min(t0, a0)
    ev.sort()
    print("%-60s %6s %9s %9s %9s" % ("kernel (K) / host call (H)", "queue", "start_us", "end_us", "dur_us"))
    for s, e, n, q in ev:
        print("%-60s %6s %9.1f %9.1f %9.1f" % (n[:60], q, (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))
    print("kernels: first start %.1f us, last end %.1f us (from the opening synchronize when the API trace is present)"
          % ((int(seg[0]["Start_Timestamp"]) - t0) / 1e3, (t_end - t0) / 1e3))


if __name__ == "__main__":
    main()

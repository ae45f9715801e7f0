#!/usr/bin/env bash
# Round 5, session ap: per-launch durations of the bench's activation QDQ launches (kernel trace,
# no stats) to see how the rate depends on the tensor's size; then tools/studies/tile_quads_probe (1, 2, 4 quads per lane).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run qdq_trace 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/qdq_trace -o run -- python3 bench.py --no-cpu-baseline --no-dropin --enc-reps 1 --plan-reps 1 --steps 3 --warmup 1
python3 - <<'PY' > $OUT/qdq_per_launch.txt 2>&1
import csv, glob, collections
f = glob.glob("gpurun_out/qdq_trace/*kernel_trace.csv")[0]
rows = [r for r in csv.DictReader(open(f)) if "tensor_vec_kernel" in r["Kernel_Name"]]
print("columns:", list(rows[0].keys()))
def items(r):
    if "Grid_Size" in r:
        return int(r["Grid_Size"])
    return int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1)
by = collections.defaultdict(list)
for r in rows:
    by[items(r)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot_t = tot_b = 0
print("grid_items elems MB(in+out) launches median_us TB/s")
for g in sorted(by):
    d = sorted(by[g]); m = d[len(d) // 2]
    b = g * 4 * 8
    tot_t += sum(d); tot_b += b * len(d)
    print(g, g * 4, round(b / 1e6, 1), len(d), round(m / 1e3, 2), round(b / m / 1e3, 3))
print("all", round(tot_b / tot_t / 1e3, 3), "TB/s over", len(rows), "launches")
PY
rm -rf $OUT/qdq_trace
run tile_quads 300 tools/studies/tile_quads_probe
grep -h '^{' $OUT/tile_quads.log > $OUT/tile_quads_probe.jsonl

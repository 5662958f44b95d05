"""Per-(kernel, grid) duration summary of a rocprofv3 kernel trace, so that the
average for one batch size can be set beside bench.py's HIP-event figure (the
--stats summary averages every launch of a kernel, whatever its batch).

    python scripts/prof_summary.py TRACE_CSV OUT_CSV"""
import csv
import sys
from collections import defaultdict

rows = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    if not k.startswith(("qpb_", "(anonymous namespace)::qpb_")):
        continue
    grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    rows[(k, grid, int(r["Workgroup_Size_X"]))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["kernel", "grid_threads", "workgroup", "calls", "avg_us", "min_us", "max_us"])
    for (k, g, wg), v in sorted(rows.items()):
        w.writerow([k, g, wg, len(v), f"{sum(v) / len(v) / 1e3:.2f}", f"{min(v) / 1e3:.2f}", f"{max(v) / 1e3:.2f}"])
print(open(sys.argv[2]).read())

"""Per-(kernel, grid) duration summary of a rocprofv3 kernel trace, so that the
average for one batch size can be set beside bench.py's HIP-event figure (the
--stats summary averages every launch of a kernel, whatever its batch).

    python scripts/prof_summary.py TRACE_CSV OUT_CSV
    python scripts/prof_summary.py RESULTS_DB OUT_CSV [STATS_CSV]   (rocprofv3's SQLite output;
                                                                   STATS_CSV: the per-kernel --stats table)"""
import csv
import sqlite3
import sys
from collections import defaultdict


def dispatches(path):
    """(kernel, grid threads, workgroup, duration ns) of every dispatch."""
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, gx, gy, gz, wx, dur in c.execute(
                "select name, grid_x, grid_y, grid_z, workgroup_x, duration from kernels"):
            yield name, gx * gy * gz, wx, dur
        return
    for r in csv.DictReader(open(path)):
        yield (r["Kernel_Name"], int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]),
               int(r["Workgroup_Size_X"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))


rows = defaultdict(list)
per_kernel = defaultdict(list)
for k, grid, wg, dur in dispatches(sys.argv[1]):
    per_kernel[k].append(dur)
    if not k.startswith(("qpb_", "(anonymous namespace)::qpb_")):
        continue
    rows[(k, grid, wg)].append(dur)
if len(sys.argv) > 3:
    tot = sum(sum(v) for v in per_kernel.values())
    with open(sys.argv[3], "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for k, v in sorted(per_kernel.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([k, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot, min(v), max(v)])
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["kernel", "grid_threads", "workgroup", "calls", "avg_us", "min_us", "max_us"])
    for (k, g, wg), v in sorted(rows.items()):
        w.writerow([k, g, wg, len(v), f"{sum(v) / len(v) / 1e3:.2f}", f"{min(v) / 1e3:.2f}", f"{max(v) / 1e3:.2f}"])
print(open(sys.argv[2]).read())

"""Every qpb_* kernel's HBM bytes per launch from two rocprofv3 PMC passes of the same
command (FETCH_SIZE, WRITE_SIZE) -> profiles/traffic.json, keyed "<kernel>@<batch>".

    python scripts/traffic_all.py FETCH_CSV WRITE_CSV

bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB units), the MI355X_MICROARCH.md
HBM-section correction (gfx950 FETCH_SIZE counts half the bytes of coalesced reads;
WRITE_SIZE is exact for streaming stores).  The batch of a launch follows from its grid:
QPs per workgroup = 4 per wave (row and wide row forms), 1 per wave (wave form), 1 per workgroup
(tree, band), 1 per lane (lane kernels, qpb_ipm_*); groups (qpb_rowgroup*) and helper kernels
are keyed by their grid in threads ("<kernel>@grid<threads>").  bench.py reads the
entry of the kernel and batch each leg launches (traffic_for)."""
import csv
import json
import os
import sys
from collections import defaultdict


def batch_of(kname, grid, wg):
    blocks = grid // wg
    if kname.startswith("qpb_row_") or kname.startswith("qpb_rowx_"):
        return blocks * 4 * (wg // 64)
    if kname.startswith("qpb_wave_"):
        return blocks * (wg // 64)
    if kname.startswith("qpb_tree_") or kname.startswith("qpb_band_"):
        return blocks
    if kname.startswith("qpb_ipm_"):
        return grid
    return None


def per_kernel(path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if r["Counter_Name"] != counter or not k.startswith("qpb_"):
            continue
        vals[(k, int(r["Grid_Size"]), int(r["Workgroup_Size"]))].append(float(r["Counter_Value"]))
    return {key: sum(v) / len(v) for key, v in vals.items()}


def main():
    f = per_kernel(sys.argv[1], "FETCH_SIZE")
    w = per_kernel(sys.argv[2], "WRITE_SIZE")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out_path = os.path.join(root, "profiles", "traffic.json")
    data = {}
    for key in sorted(set(f) & set(w)):
        k, grid, wg = key
        b = batch_of(k, grid, wg)
        tag = f"{k}@{b}" if b is not None else f"{k}@grid{grid}"
        data[tag] = dict(kernel=k, batch=b, grid_threads=grid, workgroup=wg, fetch_kb=f[key], write_kb=w[key],
                         hbm_bytes_per_launch=(2 * f[key] + w[key]) * 1024.0)
        print(tag, round(data[tag]["hbm_bytes_per_launch"]))
    json.dump(data, open(out_path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()

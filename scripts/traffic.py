"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/traffic.json.

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 for our kernels:
FETCH_SIZE reads 1/2 of the bytes of 512-B-per-wave coalesced reads on gfx950
(MI355X_MICROARCH.md, HBM section) -- calibrated on this kernel, whose input
byte count is known exactly (2 * FETCH_SIZE == algorithmic input bytes within
2 %); WRITE_SIZE matched the output bytes exactly.

    python scripts/traffic.py FETCH_CSV WRITE_CSV BATCH [BATCH ...]

The wave, row and tree kernels (qpb_wave_*, qpb_row_*, qpb_tree_*) read their inputs with 8-B
per-lane loads, an access width the guide leaves uncalibrated; its entry is
recorded with the same formula and marked "calibrated": false.
"""
import csv
import json
import os
import sys
from collections import defaultdict


def grid_for(kname, wg, batch):
    """Grid size (threads) of a launch of `batch` QPs."""
    per_block = (wg // 64 if kname.startswith("qpb_wave_") else 4 * (wg // 64) if kname.startswith("qpb_row_")
                 else 1 if kname.startswith("qpb_tree_") else wg)
    return (batch + per_block - 1) // per_block * wg


def per_kernel(path, counter, batch):
    """Mean counter value over the dispatches of `batch` QPs."""
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if r["Counter_Name"] != counter or not k.startswith(("qpb_ipm", "qpb_wave", "qpb_row", "qpb_tree")):
            continue
        if int(r["Grid_Size"]) != grid_for(k, int(r["Workgroup_Size"]), batch):
            continue
        vals[k].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    fetch, write = sys.argv[1], sys.argv[2]
    out_path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "traffic.json")
    data = json.load(open(out_path)) if os.path.exists(out_path) else {}
    for batch in map(int, sys.argv[3:]):
        f = per_kernel(fetch, "FETCH_SIZE", batch)
        w = per_kernel(write, "WRITE_SIZE", batch)
        for k in f:
            if k in w:
                data[f"{k}@{batch}"] = dict(kernel=k, batch=batch, fetch_kb=f[k], write_kb=w[k],
                               hbm_bytes_per_launch=(2 * f[k] + w[k]) * 1024.0,
                               calibrated=k.startswith("qpb_ipm"))
                print(k, batch, data[f"{k}@{batch}"])
    json.dump(data, open(out_path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()

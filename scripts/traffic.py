"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/traffic.json.

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 for our kernels:
FETCH_SIZE reads 1/2 of the bytes of 512-B-per-wave coalesced reads on gfx950
(MI355X_MICROARCH.md, HBM section) -- calibrated on this kernel, whose input
byte count is known exactly (2 * FETCH_SIZE == algorithmic input bytes within
2 %); WRITE_SIZE matched the output bytes exactly.

    python scripts/traffic.py FETCH_CSV WRITE_CSV BATCH
"""
import csv
import json
import os
import sys
from collections import defaultdict


def per_kernel(path, counter, batch):
    """Mean counter value over the dispatches of `batch` QPs (grid == batch
    rounded up to whole workgroups)."""
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or "qpb_ipm" not in r["Kernel_Name"]:
            continue
        wg = int(r["Workgroup_Size"])
        if int(r["Grid_Size"]) != (batch + wg - 1) // wg * wg:
            continue
        vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    fetch, write, batch = sys.argv[1], sys.argv[2], int(sys.argv[3])
    f = per_kernel(fetch, "FETCH_SIZE", batch)
    w = per_kernel(write, "WRITE_SIZE", batch)
    out_path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "traffic.json")
    data = json.load(open(out_path)) if os.path.exists(out_path) else {}
    for k in f:
        if k in w:
            data[k] = dict(batch=batch, fetch_kb=f[k], write_kb=w[k],
                           hbm_bytes_per_launch=(2 * f[k] + w[k]) * 1024.0)
            print(k, data[k])
    json.dump(data, open(out_path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()

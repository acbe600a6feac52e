"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel, mean counter value per dispatch.

usage: python tools/pmc_summary.py <dir> [--json out.json]
FETCH_SIZE / WRITE_SIZE are reported in KB by rocprofv3; the gfx950 FETCH_SIZE correction
(x2 for wide coalesced reads, MI355X_MICROARCH.md "HBM") is applied in the `hbm_bytes` column.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    n = n.replace("void ", "").replace("mi::", "")
    return n


def collect(root):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", "?"))
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    # counter rows come per dispatch (already summed over dimensions in rocprofv3 >= 1.0)
    out = {}
    for k, d in vals.items():
        out[k] = {c: sum(v) / len(v) for c, v in d.items()}
        out[k]["_dispatches"] = max(len(v) for v in d.values())
    return out


def main():
    root = sys.argv[1]
    res = collect(root)
    for k, d in sorted(res.items()):
        if "FETCH_SIZE" in d:
            d["fetch_bytes_corrected"] = d["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in d:
            d["write_bytes"] = d["WRITE_SIZE"] * 1024
        if "fetch_bytes_corrected" in d and "write_bytes" in d:
            d["hbm_bytes"] = d["fetch_bytes_corrected"] + d["write_bytes"]
        print(k)
        for c, v in sorted(d.items()):
            print(f"    {c:28s} {v:16.1f}")
    if "--json" in sys.argv:
        json.dump(res, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()

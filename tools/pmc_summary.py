#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM bytes.

Corrections per MI355X_MICROARCH.md §HBM: counters are in KiB; on gfx950
FETCH_SIZE reports half the bytes of 16-B/lane streaming reads (doubled
here); WRITE_SIZE is exact for 16-B/lane stores.  Output: JSON with, per
kernel, the bytes per launch and per subint (nsub given on the command line).

usage: pmc_summary.py FETCH_DIR WRITE_DIR NSUB OUT.json [LABEL]
"""
import csv
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0].replace("void ", "")
    return n.replace("ppf::", "")


def load(d, counter):
    acc = defaultdict(list)
    f = os.path.join(d, "run_counter_collection.csv")
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return acc


def main():
    fdir, wdir, nsub, out = sys.argv[1:5]
    label = sys.argv[5] if len(sys.argv) > 5 else ""
    nsub = int(nsub)
    fetch = load(fdir, "FETCH_SIZE")
    write = load(wdir, "WRITE_SIZE")
    res = {"label": label, "nsub": nsub,
           "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 16-B/lane reads); WRITE_SIZE KiB x1024",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("k_"):
            continue
        fb = max(fetch.get(k, [0.0])) * 2.0
        wb = max(write.get(k, [0.0]))
        res["kernels"][k] = {"read_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                             "bytes_per_launch": fb + wb,
                             "bytes_per_subint": (fb + wb) / nsub,
                             # all launches of the run (chains such as the split
                             # scattering solve launch k_scat_sweep many times a step)
                             "launches": len(fetch.get(k, [])),
                             "bytes_all_launches": 2.0 * sum(fetch.get(k, [0.0])) +
                             sum(write.get(k, [0.0]))}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res["kernels"].items():
        print("%-22s read %.3e  write %.3e  per-subint %.4e" % (
            k, v["read_bytes_per_launch"], v["write_bytes_per_launch"], v["bytes_per_subint"]))


if __name__ == "__main__":
    main()

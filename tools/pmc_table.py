#!/usr/bin/env python3
"""Join rocprofv3 PMC passes (run_counter_collection.csv per pass dir) into one
table: one row per (kernel, dispatch order), one column per counter."""
import csv, glob, os, re, sys, collections

def load(d):
    rows = collections.OrderedDict()
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        found = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not found:
            return rows
        f = found[0]
    for r in csv.DictReader(open(f)):
        key = int(r["Dispatch_Id"])
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
        rows.setdefault(key, {"name": name})[r["Counter_Name"]] = float(r["Counter_Value"])
        rows[key]["grid"] = r.get("Grid_Size")
    return rows

base = sys.argv[1]
passes = sorted(glob.glob(os.path.join(base, "p*/")))
tables = [list(load(p).values()) for p in passes]
n = min(len(t) for t in tables if t)
merged = []
for i in range(n):
    row = {}
    for t in tables:
        if i < len(t):
            row.update(t[i])
    merged.append(row)
cols = sorted({k for r in merged for k in r} - {"name", "grid"})
print("kernel".ljust(60), " ".join(c[:22].rjust(22) for c in cols))
for r in merged:
    print(r["name"][:60].ljust(60), " ".join(f"{r.get(c, float('nan')):22.4g}" for c in cols))

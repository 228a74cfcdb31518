"""Aggregate a rocprofv3 counter_collection.csv per kernel name (mean per
dispatch): python3 tools/pmc_by_kernel.py DIR [name substrings...]"""
import csv
import glob
import sys

d = sys.argv[1]
keys = sys.argv[2:]
rows = {}
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if keys and not any(k in n for k in keys):
            continue
        disp = rows.setdefault(n, {})
        c = disp.setdefault(int(r["Dispatch_Id"]), {})
        c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for n, disp in sorted(rows.items()):
    tot = {}
    for c in disp.values():
        for k, v in c.items():
            tot[k] = tot.get(k, 0.0) + v
    nd = len(disp)
    print(f"{n[:90]}  (x{nd})")
    print("   " + "  ".join(f"{k}={v / nd:.4g}" for k, v in sorted(tot.items())))

"""Median per-dispatch counter values of the kernels in one rocprofv3 --pmc
pass.  Usage: python tools/pmc_kernel.py run_counter_collection.csv [substring]"""
import collections
import csv
import statistics
import sys

rows = collections.defaultdict(dict)
for r in csv.DictReader(open(sys.argv[1])):
    if len(sys.argv) > 2 and sys.argv[2] not in r["Kernel_Name"]:
        continue
    d = rows[r["Dispatch_Id"]]
    d["name"] = r["Kernel_Name"].split("(")[0][:80]
    d["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    d[r["Counter_Name"]] = float(r["Counter_Value"])
by = collections.defaultdict(list)
for d in rows.values():
    by[d["name"]].append(d)
for name, ds in by.items():
    print(name, f"n={len(ds)}")
    for k in ds[0]:
        if k != "name":
            print(f"  {k:28s} {statistics.median(d[k] for d in ds):16.1f}")

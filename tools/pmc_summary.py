"""Per-kernel HBM bytes per launch from rocprofv3 --pmc passes.

Usage: python tools/pmc_summary.py FETCH_counter_collection.csv WRITE_counter_collection.csv out.json
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch; on gfx950 FETCH_SIZE reads
exactly half the bytes of a wide (16 B/lane) coalesced stream
(MI355X_MICROARCH.md §HBM), so it is doubled; WRITE_SIZE is exact for
16 B/lane stores.  Kernel names are shortened to 'name<targs>'."""
import collections
import csv
import json
import re
import sys


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*$", "", name)
    return name.replace("nd::", "")


def load(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name", r.get("Counter-Name")) != counter:
            continue
        acc[short(r.get("Kernel_Name", r.get("Kernel-Name", "")))].append(float(r.get("Counter_Value",
                                                                                    r.get("Counter-Value"))))
    return {k: sum(v) / len(v) for k, v in acc.items()}


fetch = load(sys.argv[1], "FETCH_SIZE")
write = load(sys.argv[2], "WRITE_SIZE")
out = {"note": "bytes per launch = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE half-count correction)",
       "kernels": {}}
for k in sorted(set(fetch) | set(write)):
    f, w = fetch.get(k, 0.0), write.get(k, 0.0)
    out["kernels"][k] = {"fetch_kib_raw": f, "write_kib": w, "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024)}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out)[:2000])
